"""The trees the GPU tests decode (spec_amd.tree_catalog) and the reference-derived ones."""
from __future__ import annotations

from spec_amd.tree_catalog import nested_struct_tree, precompiled_trees, shapes_tree  # noqa: F401


def jit_trees() -> list:
    return precompiled_trees()
