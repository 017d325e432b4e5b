"""Debug: pkg1 decode at a size, mismatching rows per column and their 64-row windows, against
the windows whose span exceeds the root group's slab (tree_decode.hip group_shape)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import spec_amd  # noqa: E402
from spec_amd import workload  # noqa: E402
from tests.tree_helpers import oracle_decode, oracle_encode  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
tree = spec_amd.pkg1_tree()
cols, heaps, rows = workload.tree_batch(tree, n, 100 + n)
ws, we = oracle_encode(tree, cols, heaps, n)
wrows, want = oracle_decode(tree, ws, we)
dev = torch.device("cuda:0")
s = torch.from_numpy(ws).to(dev)
e = torch.from_numpy(we.view(np.int64)).to(dev)
out = spec_amd.decode_tree(tree, s, e)
torch.cuda.synchronize()
got = [c.cpu().numpy() for c in out.cols]
ends = we.astype(np.int64)
starts = np.concatenate([[0], ends[:-1]])
span = 64.0 * len(ws) / n * 1.15 + 128 + 64
slab = (int(span) + 1023) & ~1023
over = set()
for w in range((n + 63) // 64):
    lo, hi = starts[w * 64], ends[min(n, w * 64 + 64) - 1]
    sb = max(lo - 64, 0) & ~15
    se = (hi + 16 + 15) & ~15
    if se - sb + 16 > slab:
        over.add(w)
print("slab", slab, "oversize windows", len(over), sorted(over)[:20])
for ci, (c, g, wv) in enumerate(zip(tree.columns, got, want)):
    g = g[: len(wv)]
    if g.shape != wv.shape:
        print(c.name, "shape", g.shape, wv.shape)
        continue
    bad = np.nonzero((g != wv).reshape(len(wv), -1).any(axis=1))[0]
    if len(bad):
        bw = sorted(set((bad // 64).tolist())) if c.table == 0 else []
        print(c.name, "bad rows", len(bad), bad[:8].tolist(), "windows", len(bw), bw[:10],
              "in-over", sum(1 for w in bw if w in over))
