"""Loader for libspec_amd.so — the HIP engine behind include/spec_amd.h.

The product path has no fallback: if the library is missing or fails to load, every
entry point raises.  Build it with `python -c "import __graft_entry__ as g; g.build()"`
or `make -C spec_amd/csrc`.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libspec_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "spec_amd.h")

SPEC_MAX_FIELDS = 1024  # include/spec_amd.h (schemas over 64 fields: chunked decode, wide encode)
SPEC_NESTED_MAX_FIELDS = 1024  # (halves over 64 fields: chunked decode, tree-encoder encode)


class SpecSpan(C.Structure):
    _fields_ = [("off", C.c_uint32), ("len", C.c_uint32)]


class SpecField(C.Structure):
    _fields_ = [("tag", C.c_uint16), ("kind", C.c_uint8), ("reserved", C.c_uint8)]


class SpecSchema(C.Structure):
    _fields_ = [("nfields", C.c_uint32), ("fields", SpecField * SPEC_MAX_FIELDS)]


class SpecNestedSchema(C.Structure):
    _fields_ = [("outer", SpecSchema), ("item", SpecSchema)]


SPEC_TREE_MAX_FIELDS = 1024
SPEC_TREE_MAX_TABLES = 128
SPEC_TREE_MAX_COLUMNS = 2048


class SpecTreeField(C.Structure):
    _fields_ = [("tag", C.c_uint16), ("kind", C.c_uint8), ("elem", C.c_uint8), ("parent", C.c_int16),
                ("reserved", C.c_uint16)]


class SpecTree(C.Structure):
    _fields_ = [("nfields", C.c_uint32), ("fields", SpecTreeField * SPEC_TREE_MAX_FIELDS)]


class SpecTreeTable(C.Structure):
    _fields_ = [("parent", C.c_int16), ("field", C.c_int16), ("rel", C.c_uint8), ("shape", C.c_uint8),
                ("first_column", C.c_uint16), ("ncolumns", C.c_uint16)]


class SpecTreeColumn(C.Structure):
    _fields_ = [("table", C.c_uint16), ("field", C.c_int16), ("role", C.c_uint8), ("kind", C.c_uint8),
                ("width", C.c_uint16)]


class SpecError(RuntimeError):
    def __init__(self, rc: int, what: str):
        self.rc = rc
        super().__init__(f"{what}: {strerror(rc)} (rc={rc}, hip={last_hip_error()})")


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"spec_amd: {LIB_PATH} not built (run make -C spec_amd/csrc)")
        L = C.CDLL(LIB_PATH)
        _declare(L)
        if L.spec_abi_version() != ABI_VERSION:
            raise RuntimeError(f"spec_amd: {LIB_PATH} has ABI version {L.spec_abi_version()}, this binding "
                               f"was written for {ABI_VERSION} (rebuild the library)")
        bad = struct_mismatches(L)
        if bad:
            raise RuntimeError(f"spec_amd: struct layout differs from {LIB_PATH}: {bad}")
        _lib = L
    return _lib


# include/spec_amd.h: SPEC_AMD_ABI_VERSION and the spec_abi_struct ids of the mirrored structs
ABI_VERSION = 2


def struct_mirrors():
    """{spec_abi_struct id: ctypes mirror} — every public struct this binding mirrors."""
    from .lz4 import Lz4Block, Lz4Content, Lz4State

    return {0: SpecSpan, 1: SpecField, 2: SpecSchema, 3: SpecNestedSchema, 4: SpecTreeField, 5: SpecTree,
            6: SpecTreeTable, 7: SpecTreeColumn, 8: Lz4Block, 9: Lz4State, 10: Lz4Content}


def struct_mismatches(L) -> list:
    """(struct id, what, ours, the library's) for every size / member offset that differs."""
    bad = []
    for which, T in struct_mirrors().items():
        if C.sizeof(T) != L.spec_struct_size(which):
            bad.append((T.__name__, "sizeof", C.sizeof(T), L.spec_struct_size(which)))
        for m, (name, _) in enumerate(T._fields_):
            if getattr(T, name).offset != L.spec_struct_offset(which, m):
                bad.append((T.__name__, name, getattr(T, name).offset, L.spec_struct_offset(which, m)))
        if L.spec_struct_offset(which, len(T._fields_)) != C.c_size_t(-1).value:
            bad.append((T.__name__, "members", len(T._fields_), "more"))
    return bad


def _declare(L):
    vp = C.c_void_p
    L.spec_abi_version.restype = C.c_int
    L.spec_kind_width.argtypes = [C.c_int]
    L.spec_strerror.restype = C.c_char_p
    L.spec_strerror.argtypes = [C.c_int]
    L.spec_last_hip_error.restype = C.c_int
    L.spec_last_hip_error.argtypes = []
    L.spec_abi_version.argtypes = []
    L.spec_struct_size.argtypes = [C.c_int]
    L.spec_struct_size.restype = C.c_size_t
    L.spec_struct_offset.argtypes = [C.c_int, C.c_int]
    L.spec_struct_offset.restype = C.c_size_t
    L.spec_decode_flat.argtypes = [C.POINTER(SpecSchema), vp, C.c_uint64, vp, C.c_uint64,
                                   C.POINTER(vp), vp, vp]
    L.spec_decode_flat_range.argtypes = [C.POINTER(SpecSchema), vp, C.c_uint64, vp, C.c_uint64, C.c_uint64,
                                         C.c_uint64, C.POINTER(vp), vp, vp]
    L.spec_decode_frames.argtypes = L.spec_decode_flat_range.argtypes
    L.spec_decode_flat_errors.argtypes = [C.POINTER(SpecSchema), vp, C.c_uint64, vp, C.c_uint64, C.POINTER(vp), vp, vp,
                                          vp]
    L.spec_frames_index.argtypes = [vp, C.c_uint64, vp, C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.spec_frames_index_device_workspace_size.argtypes = [C.c_uint64]
    L.spec_frames_index_device_workspace_size.restype = C.c_size_t
    L.spec_frames_index_device.argtypes = [vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp, vp, C.c_size_t, vp]
    L.spec_parse_messages.argtypes = [vp, C.c_uint64, vp, C.c_uint64, C.c_uint32, vp, vp, vp]
    L.spec_parse_batch.argtypes = [C.c_uint32, vp, C.c_uint64, vp, C.c_uint64, C.c_uint32, vp, vp, vp]
    L.spec_decode_flat_prepare.argtypes = [C.POINTER(SpecSchema), C.c_uint64, C.c_uint64]
    L.spec_set_jit.argtypes = [C.c_int]
    L.spec_set_jit.restype = None
    L.spec_decode_flat_jit_compile.argtypes = [C.POINTER(SpecSchema), C.c_uint64, C.c_uint64]
    L.spec_decode_flat_jit_compile.restype = C.c_longlong
    L.spec_encode_flat_jit_compile.argtypes = [C.POINTER(SpecSchema)]
    L.spec_encode_flat_jit_compile.restype = C.c_longlong
    L.spec_decode_nested_workspace_size.restype = C.c_size_t
    L.spec_decode_nested_workspace_size.argtypes = [C.c_uint64]
    L.spec_decode_nested_index.argtypes = [C.POINTER(SpecNestedSchema), vp, C.c_uint64, vp, C.c_uint64, vp,
                                           C.c_size_t, vp, vp]
    L.spec_decode_nested.argtypes = [C.POINTER(SpecNestedSchema), vp, C.c_uint64, vp, C.c_uint64,
                                     C.POINTER(vp), vp, vp, C.POINTER(vp), vp, C.c_uint64, vp, C.c_size_t, vp]
    L.spec_decode_nested_onepass.argtypes = [C.POINTER(SpecNestedSchema), vp, C.c_uint64, vp, C.c_uint64,
                                             C.POINTER(vp), vp, vp, C.POINTER(vp), vp, C.c_uint64, vp, C.c_size_t,
                                             vp, vp]
    L.spec_set_nested_mode.argtypes = [C.c_int]
    L.spec_set_nested_mode.restype = None
    L.spec_decode_nested_jit_compile.argtypes = [C.POINTER(SpecNestedSchema)]
    L.spec_decode_nested_jit_compile.restype = C.c_longlong
    L.spec_encode_nested_jit_compile.argtypes = [C.POINTER(SpecNestedSchema)]
    L.spec_encode_nested_jit_compile.restype = C.c_longlong
    L.spec_encode_nested_workspace_size.restype = C.c_size_t
    L.spec_encode_nested_workspace_size.argtypes = [C.c_uint64]
    L.spec_encode_nested.argtypes = [C.POINTER(SpecNestedSchema), C.POINTER(vp), C.POINTER(vp), C.POINTER(C.c_uint64),
                                     vp, C.POINTER(vp), C.POINTER(vp), C.POINTER(C.c_uint64), C.c_uint64, C.c_uint64,
                                     vp, C.c_uint64, vp, vp, C.c_size_t, vp, vp]
    for name in ("spec_device_free", "spec_host_free", "spec_stream_destroy", "spec_stream_sync"):
        getattr(L, name).argtypes = [vp]
    L.spec_device_alloc.argtypes = [C.c_size_t, C.POINTER(vp)]
    L.spec_host_alloc.argtypes = [C.c_size_t, C.POINTER(vp)]
    L.spec_stream_create.argtypes = [C.POINTER(vp)]
    for name in ("spec_copy_h2d", "spec_copy_d2h", "spec_copy_d2d"):
        getattr(L, name).argtypes = [vp, vp, C.c_size_t, vp]
    L.spec_encode_flat_workspace_size.restype = C.c_size_t
    L.spec_encode_flat_workspace_size.argtypes = [C.c_uint64]
    L.spec_encode_flat_size.argtypes = [C.POINTER(SpecSchema), C.POINTER(vp), C.c_uint64, vp,
                                        C.c_size_t, vp, vp]
    L.spec_encode_flat.argtypes = [C.POINTER(SpecSchema), C.POINTER(vp), C.POINTER(vp),
                                   C.POINTER(C.c_uint64), C.c_uint64, vp, C.c_uint64, vp, vp,
                                   C.c_size_t, vp, vp]
    L.spec_host_decoder_create.argtypes = [C.POINTER(SpecSchema), C.c_uint64, C.c_uint64, C.c_uint32, C.POINTER(vp)]
    L.spec_host_decoder_destroy.argtypes = [vp]
    L.spec_host_decoder_destroy.restype = None
    L.spec_host_decoder_out_bytes.argtypes = [vp, C.c_uint64]
    L.spec_host_decoder_out_bytes.restype = C.c_uint64
    L.spec_host_decoder_chunk.argtypes = [vp, C.c_uint64, C.c_uint32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.spec_host_decoder_run.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, vp]
    L.spec_lz4_frame_blocks.argtypes = [vp, C.c_uint64, vp, vp, C.c_uint64, C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
    L.spec_lz4_decompress.argtypes = [vp, C.c_uint64, vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp]
    L.spec_lz4_pack_workspace_size.argtypes = [C.c_uint64]
    L.spec_lz4_pack_workspace_size.restype = C.c_size_t
    L.spec_lz4_pack.argtypes = [vp, C.c_uint64, vp, C.c_uint64, vp, C.c_uint64, vp, vp, C.c_size_t, vp]
    L.spec_lz4_content_update.argtypes = [vp, vp, C.c_uint64, vp]
    L.spec_lz4_content_digest.argtypes = [vp, vp, vp]
    L.spec_tree_layout.argtypes = [C.POINTER(SpecTree), C.POINTER(SpecTreeTable), C.POINTER(C.c_uint32),
                                   C.POINTER(SpecTreeColumn), C.POINTER(C.c_uint32)]
    L.spec_tree_decoder_create.argtypes = [C.POINTER(SpecTree), C.POINTER(vp)]
    L.spec_tree_decoder_destroy.argtypes = [vp]
    L.spec_tree_decoder_destroy.restype = None
    L.spec_tree_decoder_index.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.POINTER(C.c_uint64), vp]
    L.spec_tree_decoder_decode.argtypes = [vp, C.POINTER(vp), vp]
    L.spec_packed_layout.argtypes = [C.POINTER(SpecSchema), C.c_uint64, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.spec_packed_layout.restype = C.c_uint64
    L.spec_shard_bounds.argtypes = [C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.spec_shard_bounds.restype = None
    L.spec_shard_bounds_bytes.argtypes = [vp, C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_uint64),
                                          C.POINTER(C.c_uint64)]
    L.spec_shard_bounds_bytes.restype = None
    L.spec_shard_set_split.argtypes = [vp, C.c_uint32]
    L.spec_shard_create.argtypes = [C.POINTER(C.c_int), C.c_int, C.POINTER(vp)]
    L.spec_shard_destroy.argtypes = [vp]
    L.spec_shard_destroy.restype = None
    L.spec_shard_ndev.argtypes = [vp]
    L.spec_shard_stream.argtypes = [vp, C.c_int]
    L.spec_shard_stream.restype = vp
    L.spec_shard_decode.argtypes = [vp, C.POINTER(SpecSchema), C.POINTER(vp), C.POINTER(C.c_uint64), C.POINTER(vp),
                                    C.POINTER(C.c_uint64), C.POINTER(vp)]
    L.spec_shard_decode_host.argtypes = [vp, C.POINTER(SpecSchema), vp, C.c_uint64, vp, C.c_uint64, C.POINTER(vp),
                                         C.POINTER(C.c_uint64)]
    L.spec_shard_gather.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(vp), C.c_int, vp]
    L.spec_shard_sync.argtypes = [vp]
    L.spec_shard_create_ex.argtypes = [C.POINTER(C.c_int), C.c_int, C.c_uint32, C.POINTER(vp)]
    L.spec_shard_has_comm.argtypes = [vp]
    L.spec_shard_rccl_version.argtypes = []
    L.spec_shard_set_chunks.argtypes = [vp, C.c_uint32]
    L.spec_shard_encode.argtypes = [vp, C.POINTER(SpecSchema), C.POINTER(vp), C.POINTER(vp), C.POINTER(vp),
                                    C.POINTER(C.c_uint64), C.POINTER(vp), C.POINTER(C.c_uint64), C.POINTER(vp),
                                    C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.spec_shard_host_prepare.argtypes = [vp, C.POINTER(SpecSchema), C.c_uint64, C.c_uint64, C.c_uint32]
    L.spec_shard_host_decoder.argtypes = [vp, C.c_int]
    L.spec_shard_host_decoder.restype = vp
    L.spec_shard_host_decode.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.POINTER(vp), C.POINTER(C.c_uint64)]
    L.spec_tree_decoder_run.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.POINTER(vp), vp, vp, vp]
    L.spec_tree_decoder_capacity.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.spec_tree_decoder_reserve.argtypes = [vp, C.POINTER(C.c_uint64)]
    L.spec_encode_nested_workspace_size_items.argtypes = [C.c_uint64, C.c_uint64]
    L.spec_encode_nested_workspace_size_items.restype = C.c_size_t
    L.spec_tree_jit_compile.argtypes = [C.POINTER(SpecTree)]
    L.spec_tree_jit_compile.restype = C.c_longlong
    L.spec_tree_decoder_index_spans.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint64, C.POINTER(C.c_uint64), vp]
    L.spec_decode_values.argtypes = [C.c_int, vp, C.c_uint64, vp, C.c_uint64, vp, vp, vp]
    L.spec_encode_tree_workspace_size.argtypes = [C.POINTER(SpecTree), C.POINTER(C.c_uint64)]
    L.spec_encode_tree_workspace_size.restype = C.c_size_t
    L.spec_encode_tree.argtypes = [C.POINTER(SpecTree), C.POINTER(vp), C.POINTER(vp), C.POINTER(C.c_uint64),
                                   C.POINTER(C.c_uint64), vp, C.c_uint64, vp, vp, C.c_size_t, vp, vp]


def strerror(rc: int) -> str:
    return lib().spec_strerror(rc).decode()


def last_hip_error() -> int:
    return lib().spec_last_hip_error()


def check(rc: int, what: str):
    if rc != 0:
        raise SpecError(rc, what)


def header_symbols() -> list[str]:
    """Function names declared in include/spec_amd.h."""
    src = open(HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(spec_[a-z0-9_]+)\s*\(", src)))


def set_jit(enabled: bool):
    """Schema-specialised (hiprtc) decode kernels on/off (off = the precompiled generic kernel)."""
    lib().spec_set_jit(1 if enabled else 0)
