"""BASELINE config 5 flow with the HIP decode in every rank: world_size 2 (both ranks on cuda:0 —
the box has one GPU; gloo carries the collective), each rank decodes its contiguous shard with
spec_decode_flat straight into a packed column buffer, rank 0 gathers the packed buffers (one
collective) and compares with the oracle's decode of the whole batch, spans rebased."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_shard_gloo import _free_port, rebase_spans


def _worker(rank, world, port, n, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import spec_amd
    from oracle import oracle as O
    from spec_amd import FLAT16, workload
    from spec_amd.shard import PackedColumns, gather_packed, shard_batch

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        cols, heaps = workload.flat16(n, seed=11)
        stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
        s, e, base, (r0, r1) = shard_batch(stream, ends, world, rank)
        ds = torch.from_numpy(np.ascontiguousarray(s)).to(dev)
        de = torch.from_numpy(np.ascontiguousarray(e).view(np.int64)).to(dev)
        pc = PackedColumns(FLAT16, r1 - r0, dev)
        dec = spec_amd.Decoder(FLAT16, ds, de, cols=pc.cols, status=pc.status)
        dec()
        torch.cuda.synchronize()
        parts = gather_packed(pc.buf[: pc.nbytes], dist)
        bases = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(bases, torch.tensor([base], dtype=torch.int64))
        if rank == 0:
            want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, stream, ends, FLAT16.widths, 8)
            views = []
            for k, p in enumerate(parts):
                rk0, rk1 = n * k // world, n * (k + 1) // world
                views.append(PackedColumns(FLAT16, rk1 - rk0, "cpu", buf=p.cpu()))
            ok = True
            bad = []
            for f, fld in enumerate(FLAT16.fields):
                g = rebase_spans([v.cols[f] for v in views], bases, fld.kind.name in ("STRING", "BYTES"))
                if not np.array_equal(g, want[f]):
                    ok = False
                    bad.append(f)
            st = np.concatenate([v.status.numpy() for v in views])
            ok = ok and np.array_equal(st, wst) and not st.any()
            q.put((ok, bad))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4099, 200_003])
def test_hip_decode_shards_gather_world2(dev, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(k, 2, port, n, q)) for k in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, bad = q.get(timeout=5)
    assert ok, f"mismatching fields {bad}"
