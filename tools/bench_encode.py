"""Encode timing on one GPU: spec_encode_flat (size + scan + write) over the 1M Flat16 batch and
spec_encode_nested over 1M Nested records; HIP events on the launch stream."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spec_amd  # noqa: E402
from spec_amd import FLAT16  # noqa: E402
import bench  # noqa: E402


def main():
    n = int(os.environ.get("N", 1 << 20))
    dev = torch.device("cuda", 0)
    cols, heaps, d_cols, d_heaps, stream, ends = bench.make_batch(n, 0x5EC0DE, dev)
    enc = spec_amd.Encoder(FLAT16, n, dev)
    out = torch.empty_like(stream)
    e2 = torch.empty_like(ends)
    ms, med = bench.kernel_time_events(lambda: enc.encode_into(d_cols, d_heaps, out, e2), 30)
    size_ms, _ = bench.kernel_time_events(lambda: enc.size(d_cols), 30)
    torch.cuda.synchronize()
    ok = torch.equal(out, stream) and torch.equal(e2, ends)
    heap_bytes = sum(h.numel() for h in d_heaps.values())
    alg = n * (FLAT16.column_bytes + 8) + heap_bytes + stream.numel()
    res = {"flat": {"ms": round(ms, 4), "med": round(ms, 4), "size_pass_ms": round(size_ms, 4), "GB/s": round(alg / ms / 1e6, 1),
                    "Mmsg/s": round(n / ms / 1e3, 1), "ok": ok}}
    if len(sys.argv) > 1 and sys.argv[1] == "nested":
        res["nested"] = bench.nested_leg(n, 0x5EC0DE, dev)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
