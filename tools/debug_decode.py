"""Ad-hoc GPU debugging of the decode kernel paths (not part of the test suite)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import spec_amd
from oracle import oracle as O
from spec_amd import workload, FLAT16
from tests.gpu_helpers import oracle_encode, concat_records

dev = torch.device("cuda:0")
cols, heaps = workload.flat16(4, seed=1)
stream, ends = oracle_encode(FLAT16, cols, heaps, 4)
recs = [bytes(stream[(int(ends[i-1]) if i else 0):int(ends[i])]) for i in range(4)]

def run(recs, label):
    s, e = concat_records(recs)
    wc, ws = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, s, e, FLAT16.widths)
    got = spec_amd.decode_flat(FLAT16, torch.from_numpy(s).to(dev), torch.from_numpy(e.view(np.int64)).to(dev))
    torch.cuda.synchronize()
    gs = got.status.cpu().numpy()
    bad = [f for f in range(16) if not np.array_equal(got.cols[f].cpu().numpy(), wc[f])]
    print(label, "n", len(recs), "avg", s.size / len(recs), "status gpu", gs[:4], "oracle", ws[:4], "bad fields", bad)

run(recs[:1], "single (LDS path)")
run(recs[:1] + [b"\x00" * 60000], "single + huge (global path)")
run(recs, "four")
run([b"\x07" * 3] + recs, "shifted by 3")
