"""Per-launch decode time vs how long the GPU has been busy: K back-to-back launches timed with
one event pair, for growing warm-up."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import spec_amd  # noqa: E402
from spec_amd import FLAT16  # noqa: E402
import bench  # noqa: E402

n = 1 << 20
dev = torch.device("cuda", 0)
_, _, _, _, stream, ends = bench.make_batch(n, 0x5EC0DE, dev)
dec = spec_amd.Decoder(FLAT16, stream, ends)
s = torch.cuda.current_stream()
res = []
for rnd in range(8):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(200):
        dec()
    b.record(s)
    torch.cuda.synchronize()
    res.append(round(a.elapsed_time(b) / 200, 4))
print(json.dumps({"per_launch_ms_by_round": res}))
