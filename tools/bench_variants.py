"""Quick A/B of decode kernel variants on one GPU (device-resident Flat16 1M batch).
Prints per-variant average kernel time (HIP events) and algorithmic GB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spec_amd  # noqa: E402
from spec_amd import FLAT16  # noqa: E402
import bench  # noqa: E402


def main():
    n = int(os.environ.get("N", 1 << 20))
    dev = torch.device("cuda", 0)
    cols, heaps, d_cols, d_heaps, stream, ends = bench.make_batch(n, 0x5EC0DE, dev)
    alg = stream.numel() + n * (8 + FLAT16.column_bytes + 1)
    res = {}
    ref = None
    only_jit = len(sys.argv) > 1 and sys.argv[1] == "jit"
    for name, jit in ((("jit", True),) if only_jit else (("generic", False), ("jit", True))):
        spec_amd.set_jit(jit)
        dec = spec_amd.Decoder(FLAT16, stream, ends)
        for _ in range(5):
            dec()
        torch.cuda.synchronize()
        avg, med = bench.kernel_time_events(dec, 60)
        out = [c.clone() for c in dec.cols] + [dec.status.clone()]
        if ref is None:
            ref = out
        same = all(torch.equal(a, b) for a, b in zip(ref, out))
        res[name] = {"ms": round(avg, 5), "med": round(med, 5), "GB/s": round(alg / avg / 1e6, 1),
                     "Mmsg/s": round(n / avg / 1e3, 1), "same_as_generic": same}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
