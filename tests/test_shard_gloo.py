"""Multi-process (world_size 2, gloo, CPU) tests of the record sharding and the packed column
gather used by the multi-GPU path.  Here the oracle stands in for the decode (no GPU in this
container); tests/test_gpu_shard.py runs the same flow with the HIP decode in every rank."""
from __future__ import annotations

import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from spec_amd.shard import gather_columns, gather_packed, shard_batch, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rebase_spans(parts, bases, kind_is_span):
    """Concatenate per-rank column parts; shard-relative spans of non-empty values get their
    shard's byte base added (what a consumer of config 5's gathered columns does)."""
    if not kind_is_span:
        return np.concatenate([p.numpy() if isinstance(p, torch.Tensor) else p for p in parts])
    fixed = []
    for k, p in enumerate(parts):
        a = (p.numpy() if isinstance(p, torch.Tensor) else p).view(np.uint32).copy()
        a[:, 0] += np.where(a[:, 1] > 0, np.uint32(int(bases[k])), np.uint32(0))
        fixed.append(a.view(np.uint8))
    return np.concatenate(fixed)


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle as O
    from spec_amd import FLAT16, workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1001
        cols, heaps = workload.flat16(n, seed=3)
        stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
        s, e, base, (r0, r1) = shard_batch(stream, ends, world, rank)
        dec, st = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, s, e, FLAT16.widths)
        got = gather_columns([torch.from_numpy(c) for c in dec] + [torch.from_numpy(st).reshape(-1, 1)], dist)
        bases = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(bases, torch.tensor([base], dtype=torch.int64))
        # unequal sizes and an empty rank through the packed gather
        mine = torch.arange(rank * 7, dtype=torch.int64).to(torch.uint8)
        packed = gather_packed(mine, dist)
        empty = gather_columns([], dist)
        if rank == 0:
            want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, stream, ends, FLAT16.widths)
            ok = True
            for f, fld in enumerate(FLAT16.fields):
                g = rebase_spans(got[f], bases, fld.kind.name in ("STRING", "BYTES"))
                ok = ok and np.array_equal(g, want[f])
            ok = ok and np.array_equal(np.concatenate([p.numpy().ravel() for p in got[16]]), wst)
            ok = ok and [p.numel() for p in packed] == [k * 7 for k in range(world)]
            ok = ok and all(torch.equal(p, torch.arange(k * 7).to(torch.uint8)) for k, p in enumerate(packed))
            ok = ok and empty == []
            q.put(ok)
    finally:
        dist.destroy_process_group()


def test_shard_bounds_cover():
    for n in (0, 1, 7, 1000, 16 << 20):
        for world in (1, 2, 3, 8):
            b = [shard_bounds(n, world, k) for k in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[k][1] == b[k + 1][0] for k in range(world - 1))
            assert max(r1 - r0 for r0, r1 in b) - min(r1 - r0 for r0, r1 in b) <= 1


def test_shard_and_gather_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(k, 2, port, q)) for k in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_packed_columns_aligned():
    """Every packed column starts on a 256-byte boundary (the decode kernels store 4/8/16-byte
    elements; odd shard sizes such as 2049 records must not misalign the later columns)."""
    from spec_amd import FLAT16
    from spec_amd.shard import PACK_ALIGN, PackedColumns

    for n in (0, 1, 2049, 2050, 100_003):
        pc = PackedColumns(FLAT16, n, "cpu")
        base = pc.buf.data_ptr()
        if n == 0:  # empty views have no storage pointer
            assert pc.nbytes == 0 and all(c.numel() == 0 for c in pc.cols)
            continue
        assert all((c.data_ptr() - base) % PACK_ALIGN == 0 for c in pc.cols)
        assert (pc.status.data_ptr() - base) % PACK_ALIGN == 0
        assert pc.nbytes == PackedColumns.nbytes_for(FLAT16, n) >= n * (FLAT16.column_bytes + 1)
        assert [tuple(c.shape) for c in pc.cols] == [(n, w) for w in FLAT16.widths]
        ends = [c.data_ptr() - base + c.numel() for c in pc.cols]
        assert all(e <= s for e, s in zip(ends, [c.data_ptr() - base for c in pc.cols[1:]] + [pc.status.data_ptr() - base]))


def test_packed_layout_matches_c_abi():
    """spec_amd.shard.PackedColumns and the C ABI's spec_packed_layout (what spec_shard_decode
    writes) lay the packed buffer out identically; spec_shard_bounds == shard_bounds."""
    import ctypes as C

    import spec_amd
    from spec_amd import FLAT16, Kind, Schema
    from spec_amd.shard import packed_layout

    L = spec_amd.lib()
    for schema in (FLAT16, Schema([(1, Kind.BOOL), (9, Kind.BIN256), (3, Kind.INT16)])):
        for n in (0, 1, 2049, 1 << 21):
            offs = (C.c_uint64 * 64)()
            soff = C.c_uint64()
            total = L.spec_packed_layout(C.byref(schema.c), n, offs, C.byref(soff))
            po, ps, pt = packed_layout(schema.widths, n)
            assert (list(offs[: len(schema)]), soff.value, total) == (po, ps, pt)
    for n in (0, 7, 16 << 20):
        for world in (1, 3, 8):
            for k in range(world):
                r0, r1 = C.c_uint64(), C.c_uint64()
                L.spec_shard_bounds(n, world, k, C.byref(r0), C.byref(r1))
                assert (r0.value, r1.value) == shard_bounds(n, world, k)


def _bytes_split_ref(ends, world):
    """spec_shard_bounds_bytes restated: split point j = the record boundary nearest to byte
    quantile total * j / world (ties to the later boundary's lower side: fewer bytes before)."""
    n = len(ends)
    cuts = [0]
    for j in range(1, world):
        q = int(ends[-1]) * j // world if n else 0
        i = int(np.searchsorted(ends, q, side="left")) if n else 0
        if i >= n:
            cuts.append(n)
            continue
        below = int(ends[i - 1]) if i else 0
        cuts.append(i + 1 if int(ends[i]) - q <= q - below else i)
    cuts.append(n)
    return cuts


def test_shard_bounds_bytes():
    """spec_shard_bounds_bytes (C ABI, host code): contiguous, covering, monotonic shards whose
    bytes differ from total/world by at most one record's size; equal to the restatement above;
    a skewed batch (10x record sizes, the long ones first) balances where the record split does
    not; degenerate inputs (no records, one record, more shards than records, zero-size
    records)."""
    import ctypes as C

    import spec_amd

    L = spec_amd.lib()
    rng = np.random.default_rng(9)
    sizes_long = rng.integers(2000, 2600, 20_000)
    sizes_short = rng.integers(200, 260, 180_000)
    cases = [np.cumsum(np.concatenate([sizes_long, sizes_short])).astype(np.uint64),
             np.cumsum(rng.integers(0, 300, 10_001)).astype(np.uint64),
             np.zeros(0, np.uint64), np.array([5], np.uint64), np.array([0, 0, 0], np.uint64),
             np.cumsum(np.full(5, 10)).astype(np.uint64)]
    for ends in cases:
        ends = np.ascontiguousarray(ends)
        n = len(ends)
        for world in (1, 2, 3, 8, 16):
            got = []
            for k in range(world):
                r0, r1 = C.c_uint64(), C.c_uint64()
                L.spec_shard_bounds_bytes(ends.ctypes.data if n else None, n, world, k, C.byref(r0), C.byref(r1))
                got.append((r0.value, r1.value))
            cuts = _bytes_split_ref(ends, world)
            assert got == list(zip(cuts[:-1], cuts[1:])), (n, world)
            assert got[0][0] == 0 and got[-1][1] == n
            assert all(a[1] == b[0] and a[0] <= a[1] for a, b in zip(got, got[1:] + [(n, n)]))
            if n > 100:
                sz = np.diff(np.concatenate([[0], ends.astype(np.int64)]))
                tot = int(ends[-1])
                for r0, r1 in got:
                    b = (int(ends[r1 - 1]) if r1 else 0) - (int(ends[r0 - 1]) if r0 else 0)
                    assert abs(b - tot / world) <= sz.max(), (world, b, tot / world)
    skew = cases[0]
    r1 = C.c_uint64()
    L.spec_shard_bounds_bytes(skew.ctypes.data, len(skew), 3, 0, None, C.byref(r1))
    assert abs(int(skew[r1.value - 1]) - int(skew[-1]) / 3) < 0.01 * int(skew[-1]) / 3
    assert int(skew[len(skew) // 3 - 1]) > 0.6 * int(skew[-1])  # the record split
