"""Shared helpers of the schema-tree tests: the oracle's view of a spec_amd.Tree, and comparisons
of decoded tables (spans compared by the bytes they point at where buffers differ)."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O  # noqa: F401
from oracle.tree_oracle import as_list, mismatches, oracle_decode, oracle_encode, oracle_fields  # noqa: F401
from spec_amd.schema import Kind
from spec_amd.tree import (ROLE_BEGIN, ROLE_ERRMASK, ROLE_PRESENT, ROLE_STATUS, ROLE_TYPE, ROLE_VALUE, ListOf, Message,
                           Struct, Tree)

SPAN_KINDS = (Kind.STRING, Kind.BYTES, Kind.ANY)


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




from tests.trees import nested_struct_tree, shapes_tree  # noqa: E402,F401  (trees used by the tests)
