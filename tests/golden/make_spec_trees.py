"""Writes tests/golden/spec_trees.json (and spec_amd/data/reference_trees.json, the package's
copy of the four trees the engine precompiles): the schema trees spec_amd.specfile derives from the
reference's own .spec files (run here, where /root/reference exists; the GPU box has only the
JSON).  Each entry is the flattened tree [(path, tag, kind, elem, parent), ...] of one message —
derived descriptors (tags, kinds, nesting), not the schema text.

    python tests/golden/make_spec_trees.py [/root/reference]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from spec_amd import specfile  # noqa: E402

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"

# (name, files relative to REF, import root relative to REF, package, message)
CASES = [
    ("pkg1.Message", ["internal/tests/pkg1/pkg1.spec", "internal/tests/pkg1/enum.spec",
                      "internal/tests/pkg2/submessage.spec", "internal/tests/pkg3/pkg3a/struct.spec"],
     "internal/tests", "pkg1", "Message"),
    ("pmpx.Message", ["proto/pmpx/mpx.spec"], "proto", "pmpx", "Message"),
    ("pmpx.ChannelOpen", ["proto/pmpx/mpx.spec"], "proto", "pmpx", "ChannelOpen"),
    ("prpc.Message", ["proto/prpc/rpc.spec"], "proto", "prpc", "Message"),
    ("pkg4.In", ["internal/tests/pkg4/service.spec"], "internal/tests", "pkg4", "In"),
]


def trees(ref):
    out = {}
    for name, files, root, pkg, msg in CASES:
        s = specfile.load_files([os.path.join(ref, f) for f in files], root=os.path.join(ref, root))
        out[name] = s.tree(msg, pkg).to_fields()
    return out


if __name__ == "__main__":
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "spec_trees.json")
    t = trees(REF)
    json.dump(t, open(dst, "w"), indent=0)
    print(dst)
    # the package's copy of the trees the engine precompiles (spec_amd.tree_catalog)
    from spec_amd.tree_catalog import REFERENCE_TREE_NAMES, REFERENCE_TREES_JSON

    json.dump({k: t[k] for k in REFERENCE_TREE_NAMES}, open(REFERENCE_TREES_JSON, "w"), indent=0)
    print(REFERENCE_TREES_JSON)
