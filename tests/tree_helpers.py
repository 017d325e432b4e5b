"""Shared helpers of the schema-tree tests: the oracle's view of a spec_amd.Tree, and comparisons
of decoded tables (spans compared by the bytes they point at where buffers differ)."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from spec_amd.schema import Kind
from spec_amd.tree import (ROLE_BEGIN, ROLE_ERRMASK, ROLE_PRESENT, ROLE_STATUS, ROLE_TYPE, ROLE_VALUE, ListOf, Message,
                           Struct, Tree)

SPAN_KINDS = (Kind.STRING, Kind.BYTES, Kind.ANY)


def oracle_fields(tree: Tree) -> np.ndarray:
    return O.tree_fields([(f.tag, int(f.kind), int(f.elem), f.parent) for f in tree.fields])


def as_list(tree: Tree, d: dict, fill=None):
    return [d.get(c.name, fill) for c in tree.columns]


def oracle_encode(tree: Tree, cols: dict, heaps: dict, n: int):
    return O.encode_tree_batch(oracle_fields(tree), as_list(tree, cols), as_list(tree, heaps), n)


def oracle_decode(tree: Tree, stream, ends):
    return O.decode_tree_batch(oracle_fields(tree), stream, ends)


def span_bytes(col: np.ndarray, buf: np.ndarray):
    sp = np.ascontiguousarray(col).view(np.uint32).reshape(-1, 2)
    return [bytes(buf[o: o + ln]) if ln else b"" for o, ln in sp]


def roundtrip_mismatches(tree: Tree, inputs: dict, heaps: dict, got: list, stream: np.ndarray):
    """Decoded columns `got` (layout order, numpy) vs the encode inputs: values, PRESENT and
    BEGIN equal; spans by their bytes; STATUS and ERRMASK all zero; an any field's TYPE = the last
    byte of its input value (0 if empty)."""
    bad = []
    for c, g in zip(tree.columns, got):
        if c.role in (ROLE_STATUS, ROLE_ERRMASK):
            if np.any(g):
                bad.append(c.name)
            continue
        if c.role == ROLE_TYPE:
            v = tree.fields[c.field].path
            want = np.array([b[-1] if b else 0 for b in span_bytes(inputs[v], heaps[v])], np.uint8)
            if not np.array_equal(np.asarray(g).reshape(-1), want):
                bad.append(c.name)
            continue
        want = inputs[c.name]
        if c.role == ROLE_VALUE and c.kind in SPAN_KINDS:
            if span_bytes(g, stream) != span_bytes(want, heaps[c.name]):
                bad.append(c.name)
        elif not np.array_equal(np.asarray(g).reshape(want.shape), want):
            bad.append(c.name)
    return bad


def mismatches(tree: Tree, got: list, want: list):
    bad = []
    for c, g, w in zip(tree.columns, got, want):
        g = np.asarray(g)
        if g.shape != w.shape or not np.array_equal(g, w):
            bad.append(c.name)
    return bad


# ---- trees used by the tests --------------------------------------------------------------

def shapes_tree() -> Tree:
    """Lists inside list items, big tags (big message tables), value lists of every width, a
    struct with string members (pkg1.spec ComplexStruct), any."""
    complex_s = Struct("ComplexStruct", [("bin64", Kind.BIN64), ("bin128", Kind.BIN128), ("bin256", Kind.BIN256),
                                         ("string", Kind.STRING)])
    leaf = Message("Leaf", [("u", 1, Kind.UINT64), ("vals", 2, ListOf(Kind.INT16)), ("c", 3, complex_s)])
    item = Message("Item", [("name", 1, Kind.STRING), ("leaves", 2, ListOf(leaf)), ("f", 3, Kind.FLOAT32),
                            ("bytes", 4, ListOf(Kind.BYTES))])
    big = Message("Big", [("a", 300, Kind.INT32), ("b", 7, Kind.BOOL), ("any", 1000, Kind.ANY)])
    root = Message("Root", [
        ("id", 1, Kind.BIN128), ("items", 2, ListOf(item)), ("big", 3, big), ("u16s", 4, ListOf(Kind.UINT16)),
        ("f64s", 5, ListOf(Kind.FLOAT64)), ("bools", 6, ListOf(Kind.BOOL)), ("cs", 7, ListOf(complex_s)),
        ("seq", 65535, Kind.INT64),
    ])
    return Tree(root)


def nested_struct_tree() -> Tree:
    """Structs inside structs (internal/lang/model/struct_field.go:57-70): a struct field of a
    message, a list of such structs, a sub-message holding one, and three levels of nesting."""
    inner = Struct("Inner", [("x", Kind.INT32), ("y", Kind.STRING)])
    mid = Struct("Mid", [("i", inner), ("f", Kind.FLOAT64), ("j", inner)])
    outer = Struct("Outer", [("a", Kind.INT32), ("in", inner), ("s", Kind.STRING)])
    deep = Struct("Deep", [("m", mid), ("b", Kind.BIN64), ("o", outer)])
    sub = Message("Sub", [("o", 1, outer), ("n", 2, Kind.UINT16)])
    root = Message("Root", [
        ("id", 1, Kind.INT64), ("outer", 2, outer), ("outers", 3, ListOf(outer)), ("sub", 4, sub),
        ("deep", 5, deep), ("deeps", 6, ListOf(deep)), ("tail", 7, Kind.STRING),
    ])
    return Tree(root)
