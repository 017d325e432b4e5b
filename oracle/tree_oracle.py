"""The oracle's view of a spec_amd.Tree (TEST INFRASTRUCTURE: the checker for the schema-tree
tests and the bench's tree check, never the thing measured): encode / decode a batch with the C
restatement (oracle/tree.c) and compare decoded tables."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O


def oracle_fields(tree) -> np.ndarray:
    return O.tree_fields([(f.tag, int(f.kind), int(f.elem), f.parent) for f in tree.fields])


def as_list(tree, d: dict, fill=None):
    return [d.get(c.name, fill) for c in tree.columns]


def oracle_encode(tree, cols: dict, heaps: dict, n: int):
    return O.encode_tree_batch(oracle_fields(tree), as_list(tree, cols), as_list(tree, heaps), n)


def oracle_decode(tree, stream, ends):
    return O.decode_tree_batch(oracle_fields(tree), stream, ends)


def mismatches(tree, got: list, want: list):
    bad = []
    for c, g, w in zip(tree.columns, got, want):
        g = np.asarray(g)
        if g.shape != w.shape or not np.array_equal(g, w):
            bad.append(c.name)
    return bad
