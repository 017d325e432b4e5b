"""BASELINE config 5 at full size: a 16,777,216-record Flat16 batch as 8 blocks of 2,097,152
records, sharded over a world-2 group (both ranks on cuda:0 — the box has one GPU; gloo carries
the collective), every block encoded and decoded with the HIP kernels, each rank's blocks decoded
into ONE packed buffer (spec_amd.shard.PackedColumns) and gathered to rank 0 with one collective
per rank.

Checks, at full size:
  * every block round-trips on the device: decoded fixed-width columns == the encoder's input
    columns, string/bytes lengths == the input lengths, all statuses 0;
  * the gathered buffers on rank 0 hold every block's rows (per-block row counts) and per-column
    checksums equal the ones each rank computed over its inputs before the gather;
  * oracle samples: the first and the last 20,000 records of every block, encoded by the oracle
    Writer == the GPU encoder's bytes, and decoded by the oracle == the gathered columns (spans
    rebased: the oracle's offsets are relative to the sample, the engine's to the block).
"""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_shard_gloo import _free_port

BLOCKS, BLOCK = 8, 1 << 21
SAMPLE = 20_000
SPAN_FIELDS = (13, 14)  # string, bytes


def _checksums(cols, heaps, n):
    """Per-column int64 sums of the expected decode (fixed-width columns as they are; string /
    bytes: their lengths), computed on the device."""
    out = []
    for f, c in enumerate(cols):
        if f in SPAN_FIELDS:
            out.append(int(c.view(torch.int32)[:, 1].to(torch.int64).sum()))
        else:
            out.append(int(c.to(torch.int64).sum()))
    return out


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import spec_amd
    from oracle import oracle as O
    from spec_amd import FLAT16, workload
    from spec_amd.shard import PackedColumns, gather_packed, shard_bounds

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        b0, b1 = shard_bounds(BLOCKS, world, rank)
        pc = PackedColumns(FLAT16, (b1 - b0) * BLOCK, dev)
        info = {"rank": rank, "blocks": [], "errors": []}
        for j, blk in enumerate(range(b0, b1)):
            cols, heaps = workload.flat16(BLOCK, seed=0x5EC0DE + 0x100 + blk)
            d_cols = [torch.from_numpy(c).to(dev) for c in cols]
            d_heaps = {f: torch.from_numpy(h).to(dev) for f, h in heaps.items()}
            stream, ends = spec_amd.encode_flat(FLAT16, d_cols, d_heaps, BLOCK)
            # oracle sample of the encoder: first and last SAMPLE records
            ends_h = ends.cpu().numpy().view(np.uint64)
            for r0 in (0, BLOCK - SAMPLE):
                ws, we = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, [c[r0:r0 + SAMPLE] for c in cols],
                                             [heaps.get(f) for f in range(16)], SAMPLE)
                base = int(ends_h[r0 - 1]) if r0 else 0
                got = stream[base: int(ends_h[r0 + SAMPLE - 1])].cpu().numpy()
                if not (np.array_equal(got, ws) and np.array_equal(ends_h[r0:r0 + SAMPLE] - np.uint64(base), we)):
                    info["errors"].append(f"block {blk}: encoder bytes != oracle at records {r0}..")
            rows = slice(j * BLOCK, (j + 1) * BLOCK)
            dec = spec_amd.Decoder(FLAT16, stream, ends, cols=[c[rows] for c in pc.cols], status=pc.status[rows])
            dec()
            torch.cuda.synchronize()
            # full-size round trip on the device
            for f in range(16):
                got = pc.cols[f][rows]
                if f in SPAN_FIELDS:
                    ok = torch.equal(got.view(torch.int32)[:, 1], d_cols[f].view(torch.int32)[:, 1])
                else:
                    ok = torch.equal(got, d_cols[f])
                if not ok:
                    info["errors"].append(f"block {blk}: field {f} does not round-trip")
            if int(pc.status[rows].ne(0).sum()):
                info["errors"].append(f"block {blk}: non-zero status")
            info["blocks"].append({"block": blk, "rows": BLOCK, "stream_bytes": int(stream.numel()),
                                   "tail_base": int(ends_h[BLOCK - SAMPLE - 1]),
                                   "sums": _checksums(d_cols, d_heaps, BLOCK)})
            del d_cols, d_heaps, stream, ends, dec
        torch.cuda.synchronize()
        parts = gather_packed(pc.buf[: pc.nbytes], dist)
        infos = [None] * world
        dist.all_gather_object(infos, info)
        if rank == 0:
            errors = [e for i in infos for e in i["errors"]]
            nblocks = 0
            for k, part in enumerate(parts):
                kb0, kb1 = shard_bounds(BLOCKS, world, k)
                blocks = infos[k]["blocks"]
                if [b["block"] for b in blocks] != list(range(kb0, kb1)) or any(b["rows"] != BLOCK for b in blocks):
                    errors.append(f"rank {k}: wrong blocks {[b['block'] for b in blocks]}")
                got = PackedColumns(FLAT16, (kb1 - kb0) * BLOCK, dev, buf=part.to(dev))
                for j, b in enumerate(blocks):
                    rows = slice(j * BLOCK, (j + 1) * BLOCK)
                    sums = _checksums([c[rows] for c in got.cols], None, BLOCK)
                    if sums != b["sums"]:
                        errors.append(f"block {b['block']}: gathered column checksums differ")
                    if int(got.status[rows].ne(0).sum()):
                        errors.append(f"block {b['block']}: gathered status non-zero")
                    # oracle decode of the block's first and last records vs the gathered rows
                    cols, heaps = workload.flat16(BLOCK, seed=0x5EC0DE + 0x100 + b["block"])
                    for r0 in (0, BLOCK - SAMPLE):
                        ws, we = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, [c[r0:r0 + SAMPLE] for c in cols],
                                                     [heaps.get(f) for f in range(16)], SAMPLE)
                        want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, ws, we, FLAT16.widths, 8)
                        g0 = j * BLOCK + r0
                        # the engine's spans are block-relative: rebase by the sample's byte base
                        first_off = b["tail_base"] if r0 else 0
                        for f in range(16):
                            g = got.cols[f][g0:g0 + SAMPLE].cpu().numpy()
                            if f in SPAN_FIELDS:
                                g = g.view(np.uint32).copy()
                                g[:, 0] -= np.where(g[:, 1] > 0, np.uint32(first_off), np.uint32(0))
                                g = g.view(np.uint8)
                            if not np.array_equal(g, want[f]):
                                errors.append(f"block {b['block']} records {r0}..: field {f} != oracle")
                        if not np.array_equal(got.status[g0:g0 + SAMPLE].cpu().numpy(), wst):
                            errors.append(f"block {b['block']} records {r0}..: status != oracle")
                    nblocks += 1
            if nblocks != BLOCKS:
                errors.append(f"{nblocks} blocks gathered")
            q.put(errors)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_config5_full_size_world2():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(k, 2, port, q)) for k in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    errors = q.get(timeout=5)
    assert not errors, errors[:10]
