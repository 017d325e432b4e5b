"""Nested (config 4) decode and encode timing on one GPU: one-pass and two-pass decode and the
encode, per launch (HIP events).  Prints one JSON line.  Also the command profiled for the
nested kernels' rocprofv3 stats and PMC passes (tools/gpu_round.sh)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spec_amd  # noqa: E402
from spec_amd import NESTED, workload  # noqa: E402
import bench  # noqa: E402


def main():
    n = int(os.environ.get("N", 1 << 20))
    dev = torch.device("cuda", 0)
    w = workload.nested(n, workload.SEED)
    m = len(w["key"])
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    outer = [to(w["id"]), to(w["seq"].view(np.uint8).reshape(n, 8)), to(w["name"].view(np.uint8).reshape(n, 8)), None]
    items = [to(w["key"].view(np.uint8).reshape(m, 4)), to(w["value"].view(np.uint8).reshape(m, 8)),
             to(w["label"].view(np.uint8).reshape(m, 8))]
    oh, ih, ib = {2: to(w["name_heap"])}, {2: to(w["label_heap"])}, to(w["item_begin"].view(np.int32))
    stream, ends = spec_amd.encode_nested(NESTED, outer, oh, ib, items, ih, n)
    d = spec_amd.NestedDecoder(NESTED, stream, ends)
    d.index()
    d.reserve(int(d.total.item()))

    def two():
        d.index()
        d.decode()

    res = {}
    enc = spec_amd.NestedEncoder(NESTED, n, dev)
    out = torch.empty_like(stream)
    e2 = torch.empty_like(ends)
    enc_ms, _ = bench.kernel_time_events(lambda: enc.encode(outer, oh, ib, items, ih, m, out, e2), 10)
    two_ms, _ = bench.kernel_time_events(two, 20)
    L = spec_amd.lib()
    modes = {}
    ref_items = [c.clone() for c in d.items]
    for mode, name in ((1, "groups"), (2, "ranges"), (3, "halves"), (4, "tailcount"), (5, "xcd")):
        L.spec_set_nested_mode(mode)
        for c in d.items:
            c.zero_()
        dec_ms, _ = bench.kernel_time_events(d.decode, 20)
        idx_ms, _ = bench.kernel_time_events(d.index, 20)
        both_ms, _ = bench.kernel_time_events(two, 20)
        torch.cuda.synchronize()
        same = all(torch.equal(a_, b_) for a_, b_ in zip(d.items, ref_items)) and int(d.status.sum()) == 0
        modes[name] = {"decode_ms": round(dec_ms, 4), "index_ms": round(idx_ms, 4), "twopass_ms": round(both_ms, 4),
                       "same": bool(same)}
    L.spec_set_nested_mode(5)
    res["modes"] = modes
    one_ms, _ = bench.kernel_time_events(d.decode_onepass, 20)
    torch.cuda.synchronize()
    ok = int(d.total.item()) == m and torch.equal(d.items[0], items[0]) and torch.equal(d.item_begin, ib)
    ok = ok and torch.equal(out, stream)
    res["nested"] = {"onepass_ms": round(one_ms, 4), "twopass_ms": round(two_ms, 4), "encode_ms": round(enc_ms, 4),
                     "ok": bool(ok), "med": round(one_ms, 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
