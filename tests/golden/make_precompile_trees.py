"""Writes tests/golden/precompile_trees.json: the build-time list of the test-only schema trees
(tests/trees.py extra_trees) whose schema-specialised kernels build() precompiles besides the
product's own (spec_amd.tree_catalog.product_trees), as flattened descriptors
[(path, tag, kind, elem, parent), ...].  tests/test_tree.py checks the file is current.

    python tests/golden/make_precompile_trees.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from spec_amd.tree_catalog import EXTRA_TREES_JSON  # noqa: E402
from tests.trees import extra_trees  # noqa: E402

if __name__ == "__main__":
    json.dump({k: t.to_fields() for k, t in extra_trees().items()}, open(EXTRA_TREES_JSON, "w"), indent=0)
    print(EXTRA_TREES_JSON)
