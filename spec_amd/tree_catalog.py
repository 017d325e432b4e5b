"""Schema trees the engine precompiles (build(): their schema-specialised kernels go into the
code-object cache that travels with the library): the bench's pkg1.spec Message at depths 1-3 and
the trees spec_amd.specfile derives from the reference's own .spec files.  The trees only the
tests use live in tests/trees.py; build() adds them from the build-time list
tests/golden/precompile_trees.json (extra_trees below).  No oracle here: this is product code."""
from __future__ import annotations

import json
import os

from .tree import Tree, pkg1_tree

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# the trees spec_amd.specfile derives from the reference's own .spec files (pkg1.spec,
# proto/pmpx/mpx.spec, proto/prpc/rpc.spec), as flattened descriptors (path, tag, kind, elem,
# parent) — package data written by tests/golden/make_spec_trees.py with the test fixture
REFERENCE_TREES_JSON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "reference_trees.json")
REFERENCE_TREE_NAMES = ("pkg1.Message", "pmpx.Message", "prpc.Message", "pmpx.ChannelOpen")
# build-time list of further trees to precompile (written by tests/golden/make_precompile_trees.py
# from tests/trees.py: the shapes the GPU tests decode and encode)
EXTRA_TREES_JSON = os.path.join(_ROOT, "tests", "golden", "precompile_trees.json")


def reference_trees() -> dict:
    """{name: Tree} of the reference-derived trees the engine precompiles."""
    d = json.load(open(REFERENCE_TREES_JSON))
    return {k: Tree.from_fields(d[k]) for k in REFERENCE_TREE_NAMES}


def product_trees() -> list:
    """The bench's pkg1 trees (depths 1-3) and the reference-derived trees."""
    return [pkg1_tree(k) for k in (1, 2, 3)] + list(reference_trees().values())


def extra_trees() -> dict:
    """{name: Tree} from the build-time list (empty when the list is absent)."""
    if not os.path.exists(EXTRA_TREES_JSON):
        return {}
    d = json.load(open(EXTRA_TREES_JSON))
    return {k: Tree.from_fields(v) for k, v in d.items()}


def precompiled_trees() -> list:
    """Every tree whose schema-specialised kernels build() compiles into the code-object cache."""
    return product_trees() + list(extra_trees().values())
