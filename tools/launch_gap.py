"""Where do the microseconds between back-to-back decode launches go?  Prints per-launch time
for: events around each launch; one event pair around K queued launches; host call cost."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spec_amd  # noqa: E402
from spec_amd import FLAT16  # noqa: E402
import bench  # noqa: E402


def main():
    n = 1 << 20
    dev = torch.device("cuda", 0)
    _, _, _, _, stream, ends = bench.make_batch(n, 0x5EC0DE, dev)
    dec = spec_amd.Decoder(FLAT16, stream, ends)
    for _ in range(5):
        dec()
    torch.cuda.synchronize()
    res = {}
    avg, med = bench.kernel_time_events(dec, 40)
    res["events_each"] = round(avg, 4)
    s = torch.cuda.current_stream()
    for K in (10, 40):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(int(2e8))
        a.record(s)
        for _ in range(K):
            dec()
        b.record(s)
        torch.cuda.synchronize()
        res[f"events_around_{K}"] = round(a.elapsed_time(b) / K, 4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        dec()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    res["host_us_per_call"] = round((t1 - t0) / 200 * 1e6, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
