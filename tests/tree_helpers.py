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


from tests.jit_trees import nested_struct_tree, shapes_tree  # noqa: E402,F401  (trees used by the tests)
