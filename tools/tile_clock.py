#!/usr/bin/env python3
"""Phase times of the record-tile writer (jit.cpp gen_tile) from a measurement build
(-DSPEC_AB_TILE_CLOCK=1: each tile's workgroup leaves the wall clock (100 MHz) at its phase
boundaries in its records' B.tmask entries, the workspace's last rows[0] * 8 bytes): per phase
the median and p90 over tiles, and the tiles in flight.  Usage: python3 tools/tile_clock.py [n]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spec_amd  # noqa: E402
from spec_amd import workload  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    tree = spec_amd.pkg1_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, 7)
    dev = torch.device("cuda:0")
    dc = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in cols.items()}
    dh = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in heaps.items()}
    enc = spec_amd.TreeEncoder(tree, rows, dev)
    total = int(enc.encode(dc, dh, None, None).item())
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    ends = torch.empty(n, dtype=torch.int64, device=dev)
    for _ in range(3):
        enc.encode(dc, dh, out, ends)
    torch.cuda.synchronize()
    ws = enc.workspace.view(torch.uint8)[: enc.ws_bytes]
    tm = ws[enc.ws_bytes - ((n * 8 + 255) // 256) * 256:][: n * 8].view(torch.int64).cpu().numpy()
    t = tm.reshape(-1, 64)[: n // 64]  # (whole tiles)
    depth = [0] * len(tree.tables)
    for x in tree.tables[1:]:
        depth[x.index] = depth[x.parent] + 1
    maxd = max(depth)
    start, end = t[:, 0], t[:, 63]
    marks = [t[:, k] for k in range(0, maxd + 2)] + [end]  # start, records done, depth 1.. done, end
    out = {}
    names = ["records"] + [f"depth{k}" for k in range(1, maxd + 1)] + ["copy_out"]
    for i, nm in enumerate(names):
        d = (marks[i + 1] - marks[i]) * 10e-3  # us
        out[nm] = {"median_us": round(float(np.median(d)), 2), "p90_us": round(float(np.percentile(d, 90)), 2)}
    tot = (end - start) * 10e-3
    out["tile_us"] = {"median": round(float(np.median(tot)), 2), "p90": round(float(np.percentile(tot, 90)), 2)}
    span = (end.max() - start.min()) * 10e-3
    out["kernel_span_us"] = round(float(span), 1)
    out["tiles_in_flight_avg"] = round(float(tot.sum() / span), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
