"""The trees the GPU tests decode (spec_amd.tree_catalog) and the reference-derived ones."""
from __future__ import annotations

import os

from spec_amd.tree_catalog import nested_struct_tree, precompiled_trees, shapes_tree  # noqa: F401

SPEC_TREES_JSON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "spec_trees.json")


def jit_trees() -> list:
    return precompiled_trees(SPEC_TREES_JSON)
