"""The C-ABI library (libspec_amd.so) on the CPU: it loads, exports every function
include/spec_amd.h declares, and validates arguments before touching the GPU.  No compute
call is made here (no GPU in this container); the parity tests are the -m gpu suite."""
from __future__ import annotations

import ctypes as C
import subprocess

import spec_amd
from spec_amd import _lib


def test_library_loads_and_exports_header():
    L = spec_amd.lib()
    syms = _lib.header_symbols()
    assert len(syms) >= 8
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert set(syms) <= exported


def test_library_has_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_struct_layouts_match_header():
    """ABI version 2 (SPEC_MAX_FIELDS / SPEC_TREE_MAX_FIELDS 64 / 256 -> 1024 grew spec_schema to
    4100 B and moved spec_nested_schema.item to offset 4100): every ctypes mirror has the
    library's sizeof and member offsets (spec_struct_size / spec_struct_offset), and the library's
    agree with a plain C program compiled here against include/spec_amd.h (gcc)."""
    import os
    import re
    import tempfile

    from spec_amd.lz4 import BLOCK_DTYPE, Lz4Block

    L = spec_amd.lib()
    assert L.spec_abi_version() == _lib.ABI_VERSION == 2
    hdr = open(_lib.HEADER_PATH).read()
    assert int(re.search(r"#define SPEC_AMD_ABI_VERSION (\d+)", hdr).group(1)) == _lib.ABI_VERSION
    for name in ("SPEC_MAX_FIELDS", "SPEC_NESTED_MAX_FIELDS", "SPEC_TREE_MAX_FIELDS", "SPEC_TREE_MAX_TABLES",
                 "SPEC_TREE_MAX_COLUMNS"):
        assert int(re.search(rf"#define {name} (\d+)", hdr).group(1)) == getattr(_lib, name), name
    assert _lib.struct_mismatches(L) == []
    assert C.sizeof(_lib.SpecSchema) == 4100 and _lib.SpecNestedSchema.item.offset == 4100
    assert C.sizeof(_lib.SpecTree) == 8196
    assert L.spec_struct_size(99) == 0 and L.spec_struct_offset(99, 0) == C.c_size_t(-1).value
    assert BLOCK_DTYPE.itemsize == C.sizeof(Lz4Block)
    assert [BLOCK_DTYPE.fields[n][1] for n in BLOCK_DTYPE.names] == [getattr(Lz4Block, n).offset for n in BLOCK_DTYPE.names]
    # an independent compile of the header (what a cgo binding sees)
    structs = {0: ("spec_span", ["off", "len"]), 1: ("spec_field", ["tag", "kind", "reserved"]),
               2: ("spec_schema", ["nfields", "fields"]), 3: ("spec_nested_schema", ["outer", "item"]),
               4: ("spec_tree_field", ["tag", "kind", "elem", "parent", "reserved"]),
               5: ("spec_tree", ["nfields", "fields"]),
               6: ("spec_tree_table", ["parent", "field", "rel", "shape", "first_column", "ncolumns"]),
               7: ("spec_tree_column", ["table", "field", "role", "kind", "width"]),
               8: ("spec_lz4_block", ["src_off", "src_len", "stored"]),
               9: ("spec_lz4_state", ["in_frame", "block_max", "flags", "content_checksum"]),
               10: ("spec_lz4_content", ["v", "total", "buf", "buffered", "started"])}
    assert len(structs) == len(_lib.struct_mirrors())
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "spec_amd.h"', "int main(void) {"]
    for which, (s, members) in structs.items():
        lines.append(f'printf("{which} -1 %zu\\n", sizeof({s}));')
        lines += [f'printf("{which} {m} %zu\\n", offsetof({s}, {f}));' for m, f in enumerate(members)]
    lines.append("return 0; }")
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "layout.c"), os.path.join(d, "layout")
        open(src, "w").write("\n".join(lines))
        subprocess.run(["gcc", "-std=c99", "-I", os.path.dirname(_lib.HEADER_PATH), src, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    for line in out.split("\n"):
        if line:
            which, m, v = (int(x) for x in line.split())
            got = L.spec_struct_size(which) if m < 0 else L.spec_struct_offset(which, m)
            assert got == v, (structs[which], m, got, v)


def test_introspection():
    L = spec_amd.lib()
    assert L.spec_abi_version() == 2
    widths = {1: 1, 2: 1, 3: 2, 4: 4, 5: 8, 6: 2, 7: 4, 8: 8, 9: 4, 10: 8, 11: 8, 12: 16, 13: 32, 14: 8, 15: 8}
    for k, w in widths.items():
        assert L.spec_kind_width(k) == w
    assert L.spec_kind_width(0) == 0 and L.spec_kind_width(99) == 0
    assert L.spec_strerror(0) == b"ok"
    assert b"workspace" in L.spec_strerror(-5)


def test_argument_validation_without_gpu():
    L = spec_amd.lib()
    # NULL schema / bad kind / oversize stream are rejected before any HIP call
    assert L.spec_decode_flat(None, None, 0, None, 1, None, None, None) == -1
    bad = _lib.SpecSchema()
    bad.nfields = 1
    bad.fields[0].tag = 1
    bad.fields[0].kind = 42
    assert L.spec_decode_flat(C.byref(bad), None, 0, None, 1, None, None, None) == -1
    s = spec_amd.FLAT16.c
    cols = (C.c_void_p * 16)(*([1] * 16))
    assert L.spec_decode_flat(C.byref(s), C.c_void_p(1), 1 << 32, C.c_void_p(1), 1, cols, None, None) == -3
    # n == 0 is a no-op
    assert L.spec_decode_flat(C.byref(s), None, 0, None, 0, None, None, None) == 0
    ws = L.spec_encode_flat_workspace_size(1000)
    assert ws >= 8
    assert L.spec_encode_flat_size(C.byref(s), cols, 1000, C.c_void_p(1), ws - 1, None, None) == -5


def test_encode_tree_requires_begin_columns_without_gpu():
    """spec_encode_tree: a list table's BEGIN column has owner rows + 1 entries, so it is required
    whenever the OWNER has rows, even when every list is empty (0 element rows); rejected before
    any HIP call."""
    from spec_amd.tree import ROLE_BEGIN, ROLE_STATUS, ListOf, Message, Tree

    L = spec_amd.lib()
    tree = Tree(Message("M", [("a", 1, spec_amd.Kind.INT32), ("l", 2, ListOf(spec_amd.Kind.INT64))]))
    rows = (C.c_uint64 * len(tree.tables))(5, 0)  # 5 records, no list elements
    nc = len(tree.columns)
    cols = (C.c_void_p * nc)()
    for c in tree.columns:
        if c.role != ROLE_STATUS:
            cols[c.index] = 1  # never dereferenced: validation fails first
    begin = next(c for c in tree.columns if c.role == ROLE_BEGIN)
    cols[begin.index] = None
    ws = L.spec_encode_tree_workspace_size(C.byref(tree.c), rows)
    total = (C.c_uint64 * 1)()
    rc = L.spec_encode_tree(C.byref(tree.c), cols, None, None, rows, None, 0, None, C.c_void_p(1), ws, C.c_void_p(C.addressof(total)), None)
    assert rc == -1


def test_schema_limits():
    import pytest

    wide = spec_amd.Schema([(i + 1, spec_amd.Kind.INT64) for i in range(1024)])  # chunked / wide kernels
    assert len(wide) == 1024
    with pytest.raises(ValueError):
        spec_amd.Schema([(i + 1, spec_amd.Kind.INT64) for i in range(1025)])
    # a nested half of more than 64 fields: chunked decode, encode through the tree encoder
    wn = spec_amd.NestedSchema([(1, spec_amd.Kind.LIST)], [(i + 1, spec_amd.Kind.INT32) for i in range(65)])
    assert len(wn.item) == 65
    with pytest.raises(ValueError):
        spec_amd.NestedSchema([(1, spec_amd.Kind.LIST)], [(i + 1, spec_amd.Kind.INT32) for i in range(1025)])


def test_jit_source_compiles_for_gfx950():
    """The schema-specialised decode kernel (jit.cpp) compiles with hiprtc for gfx950 here
    (compile only; loading needs the GPU)."""
    L = spec_amd.lib()
    s = spec_amd.FLAT16.c
    assert L.spec_decode_flat_jit_compile(C.byref(s), 256 << 20, 1 << 20) > 1000
    # no fast path: repeated tags => generic kernel, nothing compiled
    dup = spec_amd.Schema([(5, spec_amd.Kind.INT32), (5, spec_amd.Kind.INT64)])
    assert L.spec_decode_flat_jit_compile(C.byref(dup.c), 1000, 10) == 0
    # big tables (a tag > 255) and wide schemas (> 24 fields) have one (decode_core.hpp fast_wide)
    big = spec_amd.Schema([(300, spec_amd.Kind.INT32)])
    assert L.spec_decode_flat_jit_compile(C.byref(big.c), 1000, 10) > 1000
    wide = spec_amd.Schema([(i + 1, spec_amd.Kind.INT64) for i in range(64)])
    assert L.spec_decode_flat_jit_compile(C.byref(wide.c), 1000, 10) > 1000


def test_encode_jit_source_compiles_for_gfx950():
    """The schema-specialised encode kernels (jit.cpp over encode_core.hpp) compile with hiprtc."""
    L = spec_amd.lib()
    assert L.spec_encode_flat_jit_compile(C.byref(spec_amd.FLAT16.c)) > 1000
    # tags > 255 and repeated tags are fine for the encoder (big table / Writer tie order)
    odd = spec_amd.Schema([(300, spec_amd.Kind.INT32), (5, spec_amd.Kind.STRING), (5, spec_amd.Kind.BOOL)])
    assert L.spec_encode_flat_jit_compile(C.byref(odd.c)) > 1000
    many = spec_amd.Schema([(i + 1, spec_amd.Kind.INT64) for i in range(33)])
    assert L.spec_encode_flat_jit_compile(C.byref(many.c)) == 0


def test_nested_encode_jit_source_compiles_for_gfx950():
    """The schema-specialised nested encode kernels (jit.cpp over encode_nested_core.hpp:
    SpecEnc<outer> with the list hooks, SpecEnc<item>) compile with hiprtc for gfx950."""
    L = spec_amd.lib()
    assert L.spec_encode_nested_jit_compile(C.byref(spec_amd.NESTED.c)) > 1000
    # an item schema too wide for a specialised encoder: outer specialised, items generic
    wide = spec_amd.NestedSchema(
        [(1, spec_amd.Kind.INT64), (2, spec_amd.Kind.LIST)],
        [(i + 1, spec_amd.Kind.INT32) for i in range(40)])
    assert L.spec_encode_nested_jit_compile(C.byref(wide.c)) > 1000


def _header_prototypes():
    """(return type, name) of every function include/spec_amd.h declares."""
    import re

    src = open(_lib.HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    src = re.sub(r"^\s*#[^\n]*", ";", src, flags=re.M)  # preprocessor lines end a declaration
    out = []
    for m in re.finditer(r"(?:^|;|\})\s*((?:const\s+)?[A-Za-z_][\w ]*?[\s\*]+)(spec_[a-z0-9_]+)\s*\(", src):
        out.append((" ".join(m.group(1).split()), m.group(2)))
    return out


def test_ctypes_declarations_match_header():
    """Every entry point the Python host calls is declared to ctypes with argtypes, and every one
    returning a pointer or a 64-bit value has a matching restype.  ctypes' default (int argument,
    int result) truncates a 64-bit pointer: a stream or decoder handle returned as int, or a
    device pointer passed as int, is the host-side segfault class of the round-4 `nat1` crash
    (test_native_shard_decode_gather[1-plain])."""
    protos = _header_prototypes()
    names = {n for _, n in protos}
    assert set(_lib.header_symbols()) == names, set(_lib.header_symbols()) ^ names
    L = spec_amd.lib()
    wide = ("uint64_t", "size_t", "long long", "int64_t")
    bad = []
    for ret, name in protos:
        fn = getattr(L, name)
        if "*" in ret:
            if fn.restype not in (C.c_void_p, C.c_char_p) and "char" not in ret:
                bad.append((name, ret, fn.restype))
            if "char" in ret and fn.restype is not C.c_char_p:
                bad.append((name, ret, fn.restype))
        elif any(w in ret for w in wide):
            if fn.restype not in (C.c_uint64, C.c_size_t, C.c_longlong, C.c_int64, C.c_ulonglong):
                bad.append((name, ret, fn.restype))
    assert not bad, bad
    # every function the package calls has its argument types declared
    import pathlib
    import re

    used = set()
    for p in pathlib.Path(_lib.__file__).parent.glob("*.py"):
        used |= set(re.findall(r"\.(spec_[a-z0-9_]+)\(", p.read_text()))
    undeclared = sorted(n for n in used & names if getattr(L, n).argtypes is None)
    assert not undeclared, undeclared
