"""The trees the GPU tests decode: the product's precompiled trees (spec_amd.tree_catalog) and the
test-only ones (tests/trees.py)."""
from __future__ import annotations

from spec_amd.tree_catalog import product_trees
from tests.trees import extra_trees, nested_struct_tree, shapes_tree  # noqa: F401


def jit_trees() -> list:
    return product_trees() + list(extra_trees().values())
