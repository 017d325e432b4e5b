"""End-to-end (pinned host -> decode -> pinned host) rate of spec_amd.HostDecoder over the 1M
Flat16 batch for several chunk counts.  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n = 1 << 20
    _, _, _, _, stream, ends = bench.make_batch(n, 0x5EC0DE, dev)
    sh, eh = stream.cpu().pin_memory(), ends.cpu().pin_memory()
    res = {}
    for chunks in (4, 6, 8, 12, 16):
        rate, dt, _ = bench.e2e_decode(sh, eh, dev, reps=5, chunks=chunks)
        res[chunks] = {"mmsg_s": round(rate, 1), "ms": round(dt * 1e3, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
