#!/usr/bin/env python3
"""Benchmark: device-resident bulk decode of Flat16 spec messages on MI355X.

Metric (BASELINE.json): "Mmsg/s + GB/s decode (device-resident), 1M x 256B batch, 1/2/4/8
MI355X".  One step = one spec_decode_flat launch over a rank's whole batch (1M records of
~256 B by default) already resident in HBM.  N GPUs = N processes, each decoding its own shard
(records are independent: no data-path collective, weak scaling); value = records decoded by
all ranks / max-over-ranks time.  `--gpus N` without a torchrun environment starts the N rank
processes itself (spawned before anything touches a GPU).

Extra legs (keys beside the headline): BASELINE config 5 (a 16M-record batch sharded over the
ranks, decode-only and decode + one packed RCCL gather of all columns to rank 0), the generic
(non-specialised) decode kernel, encode, nested (config 4), the PCIe-inclusive end-to-end
decode from pinned host memory, the mpx frame index, LZ4, and the CPU oracle timed on the
host (rank 0, N=1 only).  Every run checks a 200k-record sample of the headline batch against
the oracle (decode columns/status and the encoder's bytes), outside the timed region.

Input generation uses numpy + this engine's GPU encoder; the oracle is only the checker and the
cpu_baseline leg.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # importing torch / spec_amd touches no GPU: the rank launcher below may still spawn

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import spec_amd  # noqa: E402
from spec_amd import FLAT16, workload  # noqa: E402

METRIC = "Mmsg/s + GB/s decode (device-resident), 1M×256B batch, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
COLUMN_BYTES = 122     # Flat16 decoded columns per record (spec_amd.FLAT16.column_bytes)
VERIFY_RECORDS = 200_000
SHARD_BLOCK = 1 << 21  # config 5: the 16M batch is 8 blocks of 2M records (one decode call each)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--records", type=int, default=1 << 20, help="records per GPU")
    p.add_argument("--seed", type=int, default=workload.SEED)
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--no-extras", action="store_true", help="skip encode / end-to-end legs")
    p.add_argument("--no-verify", action="store_true", help="skip the oracle check of a 200k-record sample")
    p.add_argument("--shard-total", type=int, default=1 << 24,
                   help="config 5: records of the batch sharded over all ranks (0 = skip the leg)")
    p.add_argument("--allow-env", action="store_true",
                   help="run even if SPEC_AMD_* variables are set (they are recorded in config.env)")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="collective backend for N>1 (gloo: rehearsal, every rank on the same GPU)")
    p.add_argument("--no-jit", action="store_true", help="generic decode kernel (no schema specialisation)")
    p.add_argument("--no-native", action="store_true", help="skip the native one-process multi-device leg")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                   help="PMC traffic per kernel (tools/pmc_traffic.py) used for roofline.traffic")
    return p.parse_args(argv)


def source_rev() -> str:
    """Hash of the engine's device and host sources (spec_amd/csrc) and its public header
    (include/): the code revision a kernel time or a PMC traffic figure belongs to."""
    import hashlib

    h = hashlib.sha1()
    for d in (os.path.join(ROOT, "spec_amd", "csrc"), os.path.join(ROOT, "include")):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".hpp", ".cpp", ".h")):
                h.update(f.encode())
                h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:12]


def spec_env():
    return {k: v for k, v in sorted(os.environ.items()) if k.startswith("SPEC_AMD_")}


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(rank, world, port, argv):
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    main(argv)


def launch_ranks(args, argv):
    """`--gpus N` outside torchrun: start N rank processes (spawn: fresh interpreters) from this
    process, which has not touched a GPU, and exit with the first failing rank's code."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(k, args.gpus, port, argv)) for k in range(args.gpus)]
    for p in procs:
        p.start()
    rc = 0
    live = list(procs)
    while live and not rc:  # poll all ranks: the first failure ends the others at once
        for p in list(live):
            p.join(timeout=0.2)
            if p.exitcode is not None:
                live.remove(p)
                if p.exitcode:
                    rc = p.exitcode
                    break
    for p in live:
        p.kill()
        p.join()
    sys.exit(rc if rc > 0 else (1 if rc else 0))


def host_cores():
    """Host cores this process may use: the affinity set, capped by a cgroup v2 CPU quota."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def dist_setup(args):
    """One process per GPU: rank/world from the torchrun (or launch_ranks) environment; backend
    "nccl" = RCCL over xGMI.  --backend gloo is a rehearsal mode for one-GPU boxes: every rank
    uses cuda:(local_rank mod device count) and the collectives go through host memory."""
    global _COLL_DEV
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        if args.backend == "gloo":
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
            _COLL_DEV = "cpu"
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            _COLL_DEV = "cuda"
        return dist, rank, world, torch.device("cuda", local)
    torch.cuda.set_device(0)
    return None, 0, 1, torch.device("cuda", 0)


_COLL_DEV = "cuda"
_RESULT_OUT = None  # multi-rank: the original stdout (fd 1 itself goes to stderr)


def device_key(dev) -> int:
    """A 63-bit key of the physical GPU this rank runs on (its UUID, else host + index)."""
    import hashlib
    import socket

    try:
        ident = str(torch.cuda.get_device_properties(dev).uuid)
    except Exception:
        ident = f"{socket.gethostname()}:{dev.index}"
    return int.from_bytes(hashlib.sha1(ident.encode()).digest()[:8], "little") >> 1


def distinct_devices(dist, dev) -> int:
    """How many physical GPUs the ranks use (a gloo rehearsal puts every rank on one)."""
    if dist is None:
        return 1
    keys = [torch.zeros(1, dtype=torch.int64, device=_COLL_DEV) for _ in range(dist.get_world_size())]
    dist.all_gather(keys, torch.tensor([device_key(dev)], dtype=torch.int64, device=_COLL_DEV))
    return len({int(k.item()) for k in keys})


def barrier(dist):
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_COLL_DEV)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_COLL_DEV)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def make_batch(n, seed, dev):
    cols, heaps = workload.flat16(n, seed)
    d_cols = [torch.from_numpy(c).to(dev) for c in cols]
    d_heaps = {f: torch.from_numpy(h).to(dev) for f, h in heaps.items()}
    stream, ends = spec_amd.encode_flat(FLAT16, d_cols, d_heaps, n)
    torch.cuda.synchronize()
    return cols, heaps, d_cols, d_heaps, stream, ends


def time_decode(dec, steps, warmup, dist):
    for _ in range(warmup):
        dec()
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(steps):
        dec()
    barrier(dist)
    return time.perf_counter() - t0


def kernel_time_events(fn, reps, lead=None, spread=False):
    """Average per-launch duration from HIP events on the launch stream: one event pair around
    `reps` back-to-back launches (an event between every launch adds ~10 us of marker/flush to
    each interval, which the kernel trace does not see), plus the median of per-launch pairs.
    `lead` untimed launches go first: the GPU is busy (and at its working clock) on them while
    the host enqueues the timed ones, so the interval measures the GPU, not host submission.
    (A spin kernel in front instead lets the chip drop its clock during the spin.)
    spread=True also returns the 10th / 90th percentiles of the per-launch pairs."""
    s = torch.cuda.current_stream()
    for _ in range(reps if lead is None else lead):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(s)
    for _ in range(reps):
        fn()
    b.record(s)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for x, y in evs:
        x.record(s)
        fn()
        y.record(s)
    torch.cuda.synchronize()
    ms = sorted(x.elapsed_time(y) for x, y in evs)
    if spread:
        return a.elapsed_time(b) / reps, ms[len(ms) // 2], ms[len(ms) // 10], ms[(9 * len(ms)) // 10]
    return a.elapsed_time(b) / reps, ms[len(ms) // 2]


def gpu_prewarm(fn, seconds=0.3):
    """Bring the GPU out of its idle clock state before any timing (MI355X idles at a low sclk;
    the first ~20 ms of launches run slower)."""
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(20):
            fn()
        torch.cuda.synchronize()


def cpu_baseline(stream_np, ends_np, seconds):
    """The oracle's per-record OpenMessageErr + 16 getters loop on host cores (test infra)."""
    import ctypes as C

    from oracle import oracle as O

    L = O.lib()
    n = len(ends_np)
    threads = host_cores()
    outc = [np.ones((n, w), np.uint8) for w in FLAT16.widths]
    st = np.ones(n, np.uint8)
    ptrs = (C.c_void_p * 16)(*[c.ctypes.data for c in outc])
    tags = np.array(FLAT16.tags, np.uint16)
    kinds = np.array(FLAT16.kinds, np.uint8)

    def run(th):
        L.so_decode_flat_batch(16, O._ptr(tags), O._ptr(kinds), O._ptr(stream_np), O._ptr(ends_np), n,
                               ptrs, O._ptr(st), th)

    res = {}
    for th in sorted({1, threads}):
        run(th)  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            run(th)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= seconds / 2:
                break
        res[th] = n * reps / dt / 1e6
    return res, threads, n


def host_cpu_model() -> str:
    """The host CPU's model name (/proc/cpuinfo), recorded next to the baseline's core count."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def _cpu_rate(fn, n, seconds):
    """Records per second of fn() (one pass over n records), repeated for ~seconds after a warm run."""
    fn()
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    return n * reps / dt / 1e6


def cpu_encode_baseline(cols, heaps, n, stream_bytes, seconds):
    """BASELINE config 3's CPU path beside the encode leg: the oracle's Writer loop
    (NewMessageWriterBuffer + 16 FieldWriter calls + Build per record, internal/bench/write_test.go:
    16-78) over the same 1M Flat16 columns, on 1 host thread and on every core (contiguous shards,
    one output buffer per thread)."""
    from oracle import oracle as O

    threads = host_cores()
    hl = [heaps.get(f) for f in range(len(FLAT16))]
    res = {}
    for th in sorted({1, threads}):
        run, _, _ = O.encode_flat_batch_mt(FLAT16.tags, FLAT16.kinds, cols, hl, n, 2 * stream_bytes + (64 << 20), th)
        res[th] = _cpu_rate(run, n, seconds / 2)
    return {"value": round(res[threads], 2), "unit": "Mmsg/s", "cores": threads, "kind": "port",
            "host_model": host_cpu_model(), "single_core_value": round(res[1], 2),
            "sample": f"{n} Flat16 records (the leg's batch) encoded repeatedly for ~{seconds / 2:.0f} s per thread "
                      f"count on {threads} host threads and on 1; C restatement of the Writer loop"}


def cpu_nested_baseline(w, stream_np, ends_np, seconds):
    """BASELINE config 4's CPU path beside the nested leg: the oracle's nested Writer loop
    (FieldWriter.List + MessageListWriter.Add/End per item, writer_list_msg.go:22-47) and its
    reader loop (OpenMessageErr + outer getters + MessageList.Len/Get + item getters,
    list_msg.go:88-92) over the same records, on 1 host thread and on every core."""
    from oracle import oracle as O

    threads = host_cores()
    n = len(ends_np)
    out = {}
    for th in sorted({1, threads}):
        enc, dec, _, _, _ = O.nested_batch_mt(w, stream_np, ends_np, 2 * stream_np.size + (64 << 20), th)
        out[th] = (_cpu_rate(enc, n, seconds / 4), _cpu_rate(dec, n, seconds / 4))
    return {"encode_value": round(out[threads][0], 2), "decode_value": round(out[threads][1], 2), "unit": "Mmsg/s",
            "cores": threads, "kind": "port", "host_model": host_cpu_model(),
            "single_core_encode_value": round(out[1][0], 2), "single_core_decode_value": round(out[1][1], 2),
            "sample": f"{n} Nested records (the leg's batch) encoded and decoded repeatedly for ~{seconds / 4:.0f} s "
                      f"each per thread count on {threads} host threads and on 1; C restatement of the reference's "
                      f"nested Writer and MessageList reader loops"}


def nested_leg(n, seed, dev, cpu_seconds=0.0):
    """BASELINE config 4: n Nested records (list<message>), GPU encode then GPU decode
    (index + decode launches), device-resident; kernel time via HIP events.  cpu_seconds > 0:
    the CPU baseline of the same records beside it (cpu_nested_baseline)."""
    from spec_amd import NESTED

    w = workload.nested(n, seed)
    m = len(w["key"])
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    outer = [to(w["id"]), to(w["seq"].view(np.uint8).reshape(n, 8)), to(w["name"].view(np.uint8).reshape(n, 8)), None]
    items = [to(w["key"].view(np.uint8).reshape(m, 4)), to(w["value"].view(np.uint8).reshape(m, 8)),
             to(w["label"].view(np.uint8).reshape(m, 8))]
    oh, ih, ib = {2: to(w["name_heap"])}, {2: to(w["label_heap"])}, to(w["item_begin"].view(np.int32))
    stream, ends = spec_amd.encode_nested(NESTED, outer, oh, ib, items, ih, n)
    torch.cuda.synchronize()
    enc = spec_amd.NestedEncoder(NESTED, n, dev)
    out = torch.empty_like(stream)
    e2 = torch.empty_like(ends)
    enc_ms, _ = kernel_time_events(lambda: enc.encode(outer, oh, ib, items, ih, m, out, e2), 10)
    d = spec_amd.NestedDecoder(NESTED, stream, ends)
    d.index()
    d.reserve(int(d.total.item()))

    def step():
        d.index()
        d.decode()

    two_ms, _ = kernel_time_events(step, 20)
    torch.cuda.synchronize()
    ok = torch.equal(out, stream) and int(d.status.sum()) == 0 and int(d.total.item()) == m
    ok = ok and len(d.items) == 3 and torch.equal(d.items[0], items[0]) and torch.equal(d.outer[1], outer[1])
    # one pass (spec_decode_nested_onepass): item columns sized from the index above
    d.item_begin.zero_()
    if d.items:
        d.items[0].zero_()
    dec_ms, _ = kernel_time_events(d.decode_onepass, 20)
    torch.cuda.synchronize()
    ok = ok and int(d.status.sum()) == 0 and int(d.total.item()) == m and int(d.item_status[:m].sum()) == 0
    # label spans: lengths equal the input's (offsets point into the stream, not the heap)
    ok = ok and len(d.items) == 3 and torch.equal(d.items[0], items[0]) and torch.equal(d.items[2][:, 4:], items[2][:, 4:])
    ok = ok and torch.equal(d.item_begin, ib)
    sb = stream.numel()
    dec_alg = sb + 8 * n + n * (16 + 8 + 8 + 1 + 4) + m * (4 + 8 + 8 + 1)
    enc_alg = n * (16 + 8 + 8 + 4) + m * (4 + 8 + 8) + int(w["name_heap"].size + w["label_heap"].size) + sb + 8 * n
    cpu = None
    if cpu_seconds > 0:
        cpu = cpu_nested_baseline(w, stream.cpu().numpy(), ends.cpu().numpy().view(np.uint64), cpu_seconds)
    return {"records": n, "items": m, "mean_record_bytes": round(sb / n, 1), "cpu_baseline": cpu,
            "decode_mmsg_s": round(n / (dec_ms * 1e-3) / 1e6, 1), "decode_ms": round(dec_ms, 4),
            "decode_gb_s": round(dec_alg / (dec_ms * 1e-3) / 1e9, 1),
            "decode_frac": round(dec_alg / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3),
            "decode_alg_bytes": int(dec_alg),
            "decode_note": "spec_decode_nested_onepass: count (per record from a 40-byte window at its end) + scan + decode "
                           "launched back to back, no host sync",
            "decode_twopass_ms": round(two_ms, 4),
            "encode_mmsg_s": round(n / (enc_ms * 1e-3) / 1e6, 1), "encode_ms": round(enc_ms, 4),
            "encode_gb_s": round(enc_alg / (enc_ms * 1e-3) / 1e9, 1),
            "encode_frac": round(enc_alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "encode_alg_bytes": int(enc_alg),
            "roundtrip_ok": bool(ok)}


def frames_leg(stream, ends, dev):
    """mpx frame index of the batch as frames ([u32 BE size][record], 1M frames): on the device
    (spec_frames_index_device, all launches, HIP events) and on one host core (spec_frames_index,
    the C walk), identical results."""
    from spec_amd.frames import frames_index, frames_index_device, make_frames_device

    import ctypes as C

    n = ends.numel()
    frames = make_frames_device(stream, ends)
    fends, used, st = frames_index_device(frames, n)
    L = spec_amd.lib()
    wsb = L.spec_frames_index_device_workspace_size(frames.numel())
    ws = torch.empty((wsb + 7) // 8, dtype=torch.int64, device=dev)
    e2 = torch.empty(n, dtype=torch.int64, device=dev)
    out = torch.zeros(3, dtype=torch.int64, device=dev)
    p = C.c_void_p

    def call():
        L.spec_frames_index_device(p(frames.data_ptr()), frames.numel(), p(e2.data_ptr()), n, p(out.data_ptr()),
                                   p(out.data_ptr() + 8), p(out.data_ptr() + 16), p(ws.data_ptr()), wsb,
                                   p(torch.cuda.current_stream().cuda_stream))

    ms, _ = kernel_time_events(call, 5, lead=2)
    host = frames.cpu().numpy()
    t0 = time.perf_counter()
    hends, hused = frames_index(host, n)
    host_ms = (time.perf_counter() - t0) * 1e3
    ok = st == 0 and used == hused == frames.numel() and np.array_equal(fends.cpu().numpy().view(np.uint64), hends)
    return {"frames": n, "bytes": int(frames.numel()), "device_ms": round(ms, 3),
            "device_gb_s": round(frames.numel() / (ms * 1e-3) / 1e9, 1), "host_1core_ms": round(host_ms, 3),
            "ok": bool(ok) and torch.equal(e2, fends),
            "note": "device: 6 launches (segment exits, group composition, chain, entries, emit, finish)"}


def lz4_leg(stream, ends, dev):
    """mpx with compression (f#4): the batch as frames in one LZ4 frame of 256 KiB blocks (oracle
    compressor, a Flush every 4096 frames), decompressed on the device (spec_lz4_decompress +
    spec_lz4_pack, HIP events, device-resident input), next to the oracle's decompression of
    the same frame on one host core."""
    import ctypes as C

    from oracle import oracle as O
    from spec_amd.frames import make_frames_device
    from spec_amd.lz4 import decompress, frame_blocks

    n = ends.numel()
    frames = make_frames_device(stream, ends).cpu().numpy()
    fe = spec_amd.frames_index(frames, n)[0]
    comp = O.lz4_frame_write(frames, list(fe[4095::4096]) + [frames.size], 256 << 10, close=False)
    blocks, used, bmax, rc = frame_blocks(comp)
    d = torch.from_numpy(comp).to(dev)
    out, sizes, status = decompress(d, blocks, bmax)
    ok = rc == 0 and out.numel() == frames.size and bool(torch.equal(out.cpu(), torch.from_numpy(frames)))
    L = spec_amd.lib()
    nb = len(blocks)
    db = torch.from_numpy(blocks.view(np.uint8).copy()).to(dev)
    slots = torch.empty(nb * bmax, dtype=torch.uint8, device=dev)
    sz = torch.empty(nb, dtype=torch.int32, device=dev)
    st = torch.empty(nb, dtype=torch.uint8, device=dev)
    o2 = torch.empty(nb * bmax, dtype=torch.uint8, device=dev)
    wsb = L.spec_lz4_pack_workspace_size(nb)
    ws = torch.empty((wsb + 7) // 8, dtype=torch.int64, device=dev)
    tot = torch.zeros(1, dtype=torch.int64, device=dev)
    p = C.c_void_p

    def call():
        s_ = p(torch.cuda.current_stream().cuda_stream)
        L.spec_lz4_decompress(p(d.data_ptr()), d.numel(), p(db.data_ptr()), nb, p(slots.data_ptr()), bmax,
                              p(sz.data_ptr()), p(st.data_ptr()), s_)
        L.spec_lz4_pack(p(slots.data_ptr()), bmax, p(sz.data_ptr()), nb, p(o2.data_ptr()), o2.numel(),
                        p(tot.data_ptr()), p(ws.data_ptr()), wsb, s_)

    ms, _ = kernel_time_events(call, 5, lead=1)
    # the frame's content checksum (xxh32 of the decompressed bytes, what lz4.Reader checks at the
    # end mark) on the device: serial over 16-byte stripes, timed once over the whole content
    from spec_amd.lz4 import ContentChecksum

    cc = ContentChecksum(dev)
    cs_ms, _ = kernel_time_events(lambda: cc.update(out), 1, lead=0)
    cc2 = ContentChecksum(dev)
    cc2.update(out)
    cs_ok = cc2.digest() == O.xxh32(frames)
    t0 = time.perf_counter()
    rc_h, host_out, _ = O.lz4_frame_read(comp, frames.size + 16)
    host_ms = (time.perf_counter() - t0) * 1e3
    return {"plain_bytes": int(frames.size), "compressed_bytes": int(comp.size), "blocks": nb,
            "device_ms": round(ms, 3), "device_gb_s": round(frames.size / (ms * 1e-3) / 1e9, 1),
            "content_checksum_ms": round(cs_ms, 3), "content_checksum_ok": bool(cs_ok),
            "host_oracle_1core_ms": round(host_ms, 1), "ok": bool(ok and rc_h == 0 and cs_ok),
            "note": "a parser wave and a copier wave per 256 KiB block: speculative next-token windows feed the serial chain, batches of 64 sequences copied while the next is parsed"}


def shard_leg(args, dist, rank, world, dev):
    """BASELINE config 5: a batch of args.shard_total Flat16 records (8 blocks of 2M, each block
    seeded on its own, so the batch is the same whatever the rank count) sharded over the ranks
    by contiguous blocks; each block is one spec_decode_flat call (its stream < 4 GiB, spans
    block-relative).  A rank's blocks decode into ONE packed buffer (columns + status), so the
    gather to rank 0 is a single collective (RCCL grouped send/recv over xGMI).  Reports
    decode-only and decode + gather, each timed max over ranks; rank 0 re-derives one record
    sample of the LAST rank's last block with the oracle and checks the gathered columns."""
    from spec_amd.shard import PackedColumns, gather_packed, shard_bounds

    total = args.shard_total
    nblocks = max(1, total // SHARD_BLOCK)
    bsz = total // nblocks
    b0, b1 = shard_bounds(nblocks, world, rank)
    mine = b1 - b0
    pc = PackedColumns(FLAT16, mine * bsz, dev)
    row = COLUMN_BYTES + 1
    decs, keep = [], []
    for j in range(mine):
        cols, heaps = workload.flat16(bsz, args.seed + 0x100 + b0 + j)
        d_cols = [torch.from_numpy(c).to(dev) for c in cols]
        d_heaps = {f: torch.from_numpy(h).to(dev) for f, h in heaps.items()}
        stream, ends = spec_amd.encode_flat(FLAT16, d_cols, d_heaps, bsz)
        del d_cols, d_heaps, cols, heaps
        # block j's columns: rows [j*bsz, (j+1)*bsz) of every packed column
        bc = [c[j * bsz:(j + 1) * bsz] for c in pc.cols]
        decs.append(spec_amd.Decoder(FLAT16, stream, ends, cols=bc, status=pc.status[j * bsz:(j + 1) * bsz]))
        keep.append((stream, ends))
    stream_bytes = sum(int(st.numel()) for st, _ in keep)

    def decode_all():
        for d in decs:
            d()

    reps = max(10, args.steps // 5)
    decode_all()
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(reps):
        decode_all()
    barrier(dist)
    wall_s = max_over_ranks(dist, (time.perf_counter() - t0) / reps)
    # HIP events on the launch stream around back-to-back steps (the rank's blocks), and each
    # block alone: the per-launch kernel times the 1M headline is compared with
    ev_ms, _ = kernel_time_events(decode_all, reps, lead=2)
    block_ms = [round(kernel_time_events(d_, 10, lead=2)[0], 4) for d_ in decs]
    dec_s = max_over_ranks(dist, ev_ms * 1e-3)
    bytes_all = sum_over_ranks(dist, float(stream_bytes))
    out = {"records_total": nblocks * bsz, "blocks": nblocks, "block_records": bsz, "ranks": world,
           "decode_ms": round(dec_s * 1e3, 3), "decode_mmsg_s": round(nblocks * bsz / dec_s / 1e6, 1),
           "decode_gb_s": round((bytes_all + nblocks * bsz * (8 + row)) / dec_s / 1e9, 1),
           "decode_wall_ms": round(wall_s * 1e3, 3), "block_kernel_ms": block_ms,
           "timing": "HIP events on the launch stream around back-to-back steps (max over ranks); "
                     "decode_wall_ms: perf_counter around the same steps incl. Python dispatch",
           "status_ok": bool(int(pc.status.ne(0).sum()) == 0)}
    if dist is None:
        out["gather"] = "n/a (one rank: the columns are already on rank 0)"
        return out
    recs = [(k1 - k0) * bsz for k0, k1 in (shard_bounds(nblocks, world, k) for k in range(world))]
    sizes = [PackedColumns.nbytes_for(FLAT16, r) for r in recs]

    def step():
        decode_all()
        return gather_packed(pc.buf[: pc.nbytes], dist, sizes=sizes)

    step()
    barrier(dist)
    t0 = time.perf_counter()
    for _ in range(reps):
        parts = step()
    barrier(dist)
    dg_s = max_over_ranks(dist, (time.perf_counter() - t0) / reps)
    out.update({"decode_gather_ms": round(dg_s * 1e3, 3), "decode_gather_mmsg_s": round(nblocks * bsz / dg_s / 1e6, 1),
                "gathered_gb_s": round(sum(recs[1:]) * row / dg_s / 1e9, 1),
                "gather": "one dist.gather of each rank's packed columns+status (RCCL grouped send/recv)"})
    if rank == 0 and not args.no_verify:
        from oracle import oracle as O

        m = 20_000
        lb = nblocks - 1  # the last block: on the last rank
        cols, heaps = workload.flat16(bsz, args.seed + 0x100 + lb)
        st, en = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, [c[:m] for c in cols],
                                     [heaps.get(f) for f in range(16)], m)
        want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, st, en, FLAT16.widths, host_cores())
        last = PackedColumns(FLAT16, recs[-1], "cpu", buf=parts[-1].cpu())
        r0 = last.n - bsz
        ok = all(np.array_equal(last.cols[f][r0:r0 + m].numpy(), want[f]) for f in range(16))
        out["gathered_sample_vs_oracle"] = bool(ok and np.array_equal(last.status[r0:r0 + m].numpy(), wst))
    return out


def native_shard_leg(args, world, devices_distinct):
    """The native multi-device path a cgo host drives (include/spec_amd.h spec_shard_*): ONE
    process, one stream + RCCL communicator per device, N = --gpus devices (weak scaling: 1M
    Flat16 records per device, the headline's per-GPU batch).  Per step, timed by the wall clock
    around `reps` back-to-back steps between spec_shard_sync calls (the devices run
    concurrently), plus HIP events on every device's shard stream:
      encode  spec_shard_encode: size passes, one host scan of the shard totals, write passes;
      decode  spec_shard_decode of every device's encoded shard into its packed buffer;
      gather  spec_shard_gather of every packed buffer to device 0 (grouped ncclSend/ncclRecv
              over xGMI; with one device the communicator is forced and the part is a send to
              itself, so the RCCL path executes);
      host    spec_shard_host_decode: the pinned host batch -> H2D / decode / D2H on every
              device at once (PCIe-inclusive, never the headline).
    On a box with fewer GPUs than N (a gloo rehearsal) the N shards share the visible GPUs
    (SPEC_SHARD_SHARED, no communicator) and `rehearsal` says so."""
    import ctypes as C

    from spec_amd import _lib
    from spec_amd.shard import NativeShard, PackedColumns

    visible = torch.cuda.device_count()
    n = args.records
    if visible >= world and devices_distinct >= world:
        devs, mode = list(range(world)), ("rccl" if world > 1 else "rccl-self")
        sh = NativeShard(devs, force_comm=True)
    else:
        devs, mode = [k % visible for k in range(world)], "shared-rehearsal"
        sh = NativeShard(devs, shared=True)
    L = _lib.lib()
    shards = []
    for k, d in enumerate(devs):
        cols, heaps = workload.flat16(n, args.seed + 0x200 + k)
        dv = torch.device("cuda", d)
        shards.append(([torch.from_numpy(c).to(dv) for c in cols], {f: torch.from_numpy(h).to(dv) for f, h in heaps.items()}, n))
        del cols, heaps
    outs, ends, totals, bases = sh.encode(FLAT16, shards)
    sh.sync()
    reps = max(20, args.steps)

    def timed(step, nrep):
        step()
        sh.sync()
        evs = []
        for k, d in enumerate(devs):
            with torch.cuda.device(d):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(sh.stream(k))
                evs.append((a, b))
        t0 = time.perf_counter()
        for _ in range(nrep):
            step()
        for k, (a, b) in enumerate(evs):
            b.record(sh.stream(k))
        sh.sync()
        wall = (time.perf_counter() - t0) / nrep
        dev_ms = max(a.elapsed_time(b) for a, b in evs) / nrep
        return wall, dev_ms

    for d in sorted(set(devs)):
        torch.cuda.synchronize(d)
    enc_wall, enc_dev = timed(sh.encode_call(FLAT16, shards, outs, ends), reps)
    # decode: every device's shard, ends relative to its own stream (prepared ctypes arguments,
    # so the timed loop is the C ABI calls alone, as a cgo caller issues them)
    rel = [(e - b).contiguous() for e, b in zip(ends, bases)]
    packs = [PackedColumns(FLAT16, n, torch.device("cuda", d)) for d in devs]
    k_ = len(devs)
    sp = (C.c_void_p * k_)(*[o.data_ptr() for o in outs])
    lens = (C.c_uint64 * k_)(*totals)
    ep = (C.c_void_p * k_)(*[e.data_ptr() for e in rel])
    ns = (C.c_uint64 * k_)(*[n] * k_)
    pp = (C.c_void_p * k_)(*[p.buf.data_ptr() for p in packs])
    for d in sorted(set(devs)):  # rel / packs come from torch's streams: complete before the shard streams use them
        torch.cuda.synchronize(d)

    def decode():
        _lib.check(L.spec_shard_decode(sh._h, C.byref(FLAT16.c), sp, lens, ep, ns, pp), "spec_shard_decode")

    dec_wall, dec_dev = timed(decode, reps)
    sizes = [p.nbytes for p in packs]
    gathered = torch.empty(sum(sizes), dtype=torch.uint8, device=torch.device("cuda", devs[0]))
    nb = (C.c_uint64 * k_)(*sizes)

    def gather():
        _lib.check(L.spec_shard_gather(sh._h, nb, pp, 0, C.c_void_p(gathered.data_ptr())), "spec_shard_gather")

    gat_wall, gat_dev = timed(gather, reps)

    def dec_gather():
        decode()
        gather()

    dg_wall, _ = timed(dec_gather, reps)
    # checks: every device's decoded fixed-width columns == its input columns, string lengths
    # equal; the gathered buffer == the packed buffers back to back; a 20k-record sample of the
    # last shard: the oracle Writer's bytes == the encoded shard, the oracle decode == its columns
    ok = int(sum(int(p.status.ne(0).sum()) for p in packs)) == 0
    for k, (p, s) in enumerate(zip(packs, shards)):
        for f in (0, 3, 4, 9, 12, 15):
            ok = ok and torch.equal(p.cols[f], s[0][f])
        ok = ok and torch.equal(p.cols[13][:, 4:], s[0][13][:, 4:])
    g = gathered.cpu()
    off = 0
    for p in packs:
        ok = ok and torch.equal(g[off:off + p.nbytes], p.buf[: p.nbytes].cpu())
        off += p.nbytes
    sample_ok = None
    if not args.no_verify:
        from oracle import oracle as O

        m = min(20_000, n)
        cols, heaps = workload.flat16(n, args.seed + 0x200 + k_ - 1)
        st, en = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, [c[:m] for c in cols], [heaps.get(f) for f in range(16)], m)
        want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, st, en, FLAT16.widths, host_cores())
        last = packs[-1]
        sample_ok = bool(np.array_equal(outs[-1][: st.size].cpu().numpy(), st)
                         and np.array_equal(rel[-1][:m].cpu().numpy(), en.view(np.int64))
                         and all(np.array_equal(last.cols[f][:m].cpu().numpy(), want[f]) for f in range(16))
                         and np.array_equal(last.status[:m].cpu().numpy(), wst))
    res = {"devices": devs, "mode": mode, "rccl_version": NativeShard.rccl_version(), "has_comm": sh.has_comm,
           "records_per_device": n, "records_total": n * k_, "stream_bytes_total": int(sum(totals)),
           "encode_ms": round(enc_wall * 1e3, 4), "encode_mmsg_s": round(n * k_ / enc_wall / 1e6, 1),
           "encode_device_ms_max": round(enc_dev, 4),
           "decode_ms": round(dec_wall * 1e3, 4), "decode_mmsg_s": round(n * k_ / dec_wall / 1e6, 1),
           "decode_device_ms_max": round(dec_dev, 4),
           "decode_device_mmsg_s": round(n * k_ / (dec_dev * 1e-3) / 1e6, 1),
           "gather_ms": round(gat_wall * 1e3, 4), "gather_bytes": int(sum(sizes)),
           "gather_gb_s": round(sum(sizes) / gat_wall / 1e9, 1),
           "decode_gather_ms": round(dg_wall * 1e3, 4), "decode_gather_mmsg_s": round(n * k_ / dg_wall / 1e6, 1),
           "columns_ok": bool(ok), "oracle_sample_ok": sample_ok}
    # host batch in, host columns out, every device at once (pinned, chunked)
    try:
        whole = torch.empty(int(sum(totals)), dtype=torch.uint8).pin_memory()
        off = 0
        for o, t in zip(outs, totals):
            whole[off:off + t].copy_(o[:t].cpu())
            off += t
        gends = torch.cat([e.cpu() for e in ends]).pin_memory()
        # the host batch split by bytes (spec_shard_bounds_bytes): every device the same bytes
        sh.set_split(True)
        N = n * k_
        bnd = [sh.bounds(N, k, gends.numpy()) for k in range(k_)]
        hb = [int(gends[r1 - 1]) - (int(gends[r0 - 1]) if r0 else 0) for r0, r1 in bnd]
        sh.host_prepare(FLAT16, max(r1 - r0 for r0, r1 in bnd), max(hb), chunks=8)
        hout = [torch.empty(sh.host_out_bytes(k, r1 - r0), dtype=torch.uint8).pin_memory()
                for k, (r0, r1) in enumerate(bnd)]
        sh.host_decode(whole, gends, hout)
        t0 = time.perf_counter()
        hreps = 3
        for _ in range(hreps):
            sh.host_decode(whole, gends, hout)
        host_s = (time.perf_counter() - t0) / hreps
        R0, R1 = bnd[-1]
        r0, r1, co, so = sh.host_chunk(k_ - 1, R1 - R0, 0)
        col4 = torch.cat([sd[0][4].reshape(-1).cpu() for sd in shards]).numpy().view(np.uint8)
        h_ok = bool(np.array_equal(hout[-1].numpy()[co[4]: co[4] + (r1 - r0) * 8],
                                   col4[(R0 + r0) * 8: (R0 + r1) * 8]))
        res.update({"host_e2e_ms": round(host_s * 1e3, 3), "host_e2e_mmsg_s": round(N / host_s / 1e6, 1),
                    "host_e2e_ok": h_ok, "host_split": "bytes", "host_shard_bytes": hb,
                    "host_note": "pinned host batch -> per device 8 chunks H2D/decode/D2H on 3 streams, devices "
                                 "on their own host threads (spec_shard_host_decode, byte-balanced shards); "
                                 "PCIe-bound"})
    except Exception as e:  # the PCIe leg never hides the device-resident numbers
        res["host_e2e_error"] = repr(e)[:300]
    del sh
    return res


def wide_leg(dev, n=1 << 20, seed=11):
    """Schemas outside the register-resident fast path (decode_core.hpp fast_wide): a 40-field
    schema (every kind, write order permuted) and a 16-field schema whose tags > 255 make every
    table big (6-byte entries, internal/format/msg.go:43-61, 138-186).  n records each, encoded
    on the GPU; the schema-specialised kernel and the generic kernel timed with HIP events; their
    columns must match each other, and a 20k-record sample the oracle."""
    from oracle import oracle as O

    schemas = workload.bench_wide_schemas()
    res = {}
    for name, sc in schemas.items():
        cols, heaps = workload.gen_columns(sc, n, seed, str_len=(0, 24))
        d_cols = [torch.from_numpy(c).to(dev) for c in cols]
        d_heaps = {f: torch.from_numpy(h).to(dev) for f, h in heaps.items()}
        stream, ends = spec_amd.encode_flat(sc, d_cols, d_heaps, n)
        del d_cols, d_heaps
        torch.cuda.synchronize()
        out = {}
        got = {}
        for jit in (True, False):
            spec_amd.set_jit(jit)
            try:
                dec = spec_amd.Decoder(sc, stream, ends)
                gpu_prewarm(dec, 0.1)
                ms, _ = kernel_time_events(dec, 20)
                torch.cuda.synchronize()
                got[jit] = dec
            finally:
                spec_amd.set_jit(True)
            col_bytes = sum(f.width for f in sc.fields)
            alg = stream.numel() + n * (8 + col_bytes + 1)
            out["jit" if jit else "generic"] = {"ms": round(ms, 4), "mmsg_s": round(n / (ms * 1e-3) / 1e6, 1),
                                                "gb_s": round(alg / (ms * 1e-3) / 1e9, 1),
                                                "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        same = torch.equal(got[True].status, got[False].status) and all(
            torch.equal(a, b) for a, b in zip(got[True].cols, got[False].cols))
        m = 20_000
        st, en = O.encode_flat_batch(sc.tags, sc.kinds, [c[:m] for c in cols], [heaps.get(f) for f in range(len(sc))], m)
        want, wst = O.decode_flat_batch(sc.tags, sc.kinds, st, en, sc.widths, host_cores())
        ok = bool(np.array_equal(got[True].status[:m].cpu().numpy(), wst) and all(
            np.array_equal(got[True].cols[f][:m].cpu().numpy(), want[f]) for f in range(len(sc))))
        out.update({"fields": len(sc), "mean_record_bytes": round(stream.numel() / n, 1),
                    "alg_bytes": int(stream.numel() + n * (8 + sum(f.width for f in sc.fields) + 1)),
                    "jit_vs_generic_same": bool(same), "oracle_sample_ok": ok})
        res[name] = out
        del got, stream, ends
    return res


def _native_child(args, world, devices, q):
    try:
        res = native_shard_leg(args, world, devices)
    except Exception as e:  # reported in the result line, never fatal
        res = {"error": repr(e)[:300]}
    q.put(res)


def native_leg_isolated(args, world, devices, timeout=300.0):
    """native_shard_leg in a fresh child process (spawned: its own HIP contexts and RCCL
    communicator), so a failure or a hang there (e.g. a communicator that never forms on some
    machine) cannot take the headline measurement with it: after `timeout` seconds the child is
    killed and the leg reports an error."""
    import multiprocessing as mp
    import queue

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_native_child, args=(args, world, devices, q))
    p.start()
    try:
        res = q.get(timeout=timeout)
    except queue.Empty:
        res = {"error": f"native leg did not finish in {timeout:.0f} s (child killed)"}
    p.join(timeout=60)
    if p.is_alive():
        p.kill()
        p.join()
    return res


def generic_leg(stream, ends, want_cols, want_status, avg_jit_ms):
    """The precompiled generic decode kernel (no schema specialisation: what schemas without a
    fast path run) on the headline batch; its columns must equal the specialised kernel's."""
    spec_amd.set_jit(False)
    try:
        dec = spec_amd.Decoder(FLAT16, stream, ends)
        gpu_prewarm(dec, 0.1)
        ms, _ = kernel_time_events(dec, 20)
        torch.cuda.synchronize()
        same = torch.equal(dec.status, want_status) and all(torch.equal(a, b) for a, b in zip(dec.cols, want_cols))
    finally:
        spec_amd.set_jit(True)
    n = ends.numel()
    alg = stream.numel() + n * (8 + COLUMN_BYTES + 1)
    return {"kernel": "decode_flat_kernel", "ms": round(ms, 4), "mmsg_s": round(n / (ms * 1e-3) / 1e6, 1),
            "gb_s": round(alg / (ms * 1e-3) / 1e9, 1), "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "vs_specialised": round(ms / avg_jit_ms, 2), "same_columns": bool(same)}


def errmask_leg(stream, ends, want_cols, want_status, avg_jit_ms):
    """spec_decode_flat_errors on the headline batch (the schema-specialised errmask variant):
    decode + a per-record uint64 of field *Err bits (internal/types/msg.go:233-459).  Same
    columns as spec_decode_flat, masks all zero (every record is a Writer's)."""
    import ctypes as C

    from spec_amd import _lib
    from spec_amd.batch import alloc_columns

    n = ends.numel()
    cols = alloc_columns(FLAT16, n, stream.device)
    st = torch.empty(n, dtype=torch.uint8, device=stream.device)
    em = torch.empty(n, dtype=torch.int64, device=stream.device)
    ptrs = (C.c_void_p * len(cols))(*[c.data_ptr() for c in cols])
    L = _lib.lib()
    args = (C.byref(FLAT16.c), C.c_void_p(stream.data_ptr()), stream.numel(), C.c_void_p(ends.data_ptr()), n, ptrs,
            C.c_void_p(st.data_ptr()), C.c_void_p(em.data_ptr()), None)

    def run():
        _lib.check(L.spec_decode_flat_errors(*args), "spec_decode_flat_errors")

    run()
    ms, _ = kernel_time_events(run, 20)
    torch.cuda.synchronize()
    same = torch.equal(st, want_status) and all(torch.equal(a, b) for a, b in zip(cols, want_cols))
    alg = stream.numel() + n * (8 + COLUMN_BYTES + 1 + 8)
    return {"ms": round(ms, 4), "mmsg_s": round(n / (ms * 1e-3) / 1e6, 1), "gb_s": round(alg / (ms * 1e-3) / 1e9, 1),
            "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "vs_decode": round(ms / avg_jit_ms, 3),
            "same_columns": bool(same), "masks_zero": bool(int((em != 0).sum().item()) == 0)}


def verify_sample(cols, heaps, stream, ends, out_cols, status, m):
    """Oracle check of the first m records, outside any timed region: the oracle Writer's bytes
    for their columns == the GPU encoder's stream prefix, and the oracle's OpenMessageErr +
    getters over those bytes == the GPU decode's columns and status."""
    from oracle import oracle as O

    m = min(m, ends.numel())
    want_stream, want_ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, [c[:m] for c in cols],
                                                 [heaps.get(f) for f in range(16)], m)
    got_stream = stream[: int(ends[m - 1])].cpu().numpy() if m else np.zeros(0, np.uint8)
    enc_ok = np.array_equal(got_stream, want_stream) and np.array_equal(
        ends[:m].cpu().numpy(), want_ends.view(np.int64))
    want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, want_stream, want_ends, FLAT16.widths, host_cores())
    dec_ok = np.array_equal(status[:m].cpu().numpy(), wst) and all(
        np.array_equal(out_cols[f][:m].cpu().numpy(), want[f]) for f in range(16))
    return {"records": m, "encode_bytes_vs_oracle": bool(enc_ok), "decode_vs_oracle": bool(dec_ok)}


def tree_leg(dev, n=1 << 18, seed=7):
    """Schema trees (the generic any-shape path): pkg1.spec's Message — structs, enum, sub-messages,
    recursive Submessage, value lists, struct lists, message lists, any — n records encoded with
    spec_encode_tree and decoded with spec_tree_decoder_* (index + decode), wall time per call
    (both synchronise with the host once per list table); encode bytes and every decoded column
    checked against the oracle outside the timed region."""
    from oracle import oracle as O  # noqa: F401  (checker only)
    from oracle.tree_oracle import mismatches, oracle_decode, oracle_encode

    tree = spec_amd.pkg1_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, seed)
    dc = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in cols.items()}
    dh = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in heaps.items()}
    enc = spec_amd.TreeEncoder(tree, rows, dev)
    total = int(enc.encode(dc, dh, None, None).item())
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    ends = torch.empty(n, dtype=torch.int64, device=dev)

    def encode():
        enc.encode(dc, dh, out, ends)

    encode()
    torch.cuda.synchronize()
    d = spec_amd.TreeDecoder(tree)
    d.index(out, ends)
    dcols = d.alloc(dev)
    rows_out = torch.empty(len(tree.tables), dtype=torch.int64, device=dev)
    col_rows = d.column_capacity(dcols)

    def decode():  # one asynchronous pass: every group kernel + list scans, no host sync
        d.run(out, ends, dcols, rows_out, col_rows=col_rows)

    res = {}
    encode()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        encode()
    torch.cuda.synchronize()
    enc_wall = (time.perf_counter() - t0) / reps
    gpu_prewarm(encode, 0.1)
    enc_ms, _ = kernel_time_events(encode, 20)
    res["encode"] = enc_ms * 1e-3
    gpu_prewarm(decode, 0.1)
    dec_ms, _ = kernel_time_events(decode, 20)
    res["decode"] = dec_ms * 1e-3
    t0 = time.perf_counter()
    d.index(out, ends)
    d.decode(cols=dcols)
    torch.cuda.synchronize()
    index_decode_s = time.perf_counter() - t0
    decode()
    torch.cuda.synchronize()
    got = spec_amd.TreeColumns(tree, list(d.rows), [c[: tree.column_rows(tc, d.rows)] for c, tc in zip(dcols, tree.columns)])
    ok_rows = [int(r) for r in rows_out.cpu()] == d.rows
    want_stream, want_ends = oracle_encode(tree, cols, heaps, n)
    ok = np.array_equal(out.cpu().numpy(), want_stream) and np.array_equal(ends.cpu().numpy().view(np.uint64), want_ends)
    wrows, want = oracle_decode(tree, want_stream, want_ends)
    ok = ok and ok_rows and wrows == got.rows and not mismatches(tree, [c.cpu().numpy() for c in got.cols], want)
    col_bytes = sum(int(c.numel()) for c in got.cols)
    alg = total + 8 * n + col_bytes  # stream + ends read, every column written
    # encode: the input columns (values, PRESENT, BEGIN) and heaps read, stream + ends written
    in_bytes = sum(int(v.numel()) for k, v in dc.items()) + sum(int(v.numel()) for v in dh.values())
    enc_alg = in_bytes + total + 8 * n
    return {"records": n, "tables": len(tree.tables), "columns": len(tree.columns), "rows": rows,
            "mean_record_bytes": round(total / n, 1), "column_bytes": col_bytes,
            "decode_ms": round(res["decode"] * 1e3, 4), "decode_mmsg_s": round(n / res["decode"] / 1e6, 1),
            "decode_gb_s": round(alg / res["decode"] / 1e9, 1),
            "decode_frac": round(alg / res["decode"] / 1e9 / HBM_PEAK_GBS, 4), "decode_alg_bytes": int(alg),
            "decode_note": "spec_tree_decoder_run: one asynchronous pass (group kernels + list scans), HIP events",
            "index_plus_decode_wall_ms": round(index_decode_s * 1e3, 3),
            "encode_ms": round(res["encode"] * 1e3, 4), "encode_mmsg_s": round(n / res["encode"] / 1e6, 1),
            "encode_gb_s": round(enc_alg / res["encode"] / 1e9, 1),
            "encode_frac": round(enc_alg / res["encode"] / 1e9 / HBM_PEAK_GBS, 4), "encode_alg_bytes": int(enc_alg),
            "encode_wall_ms": round(enc_wall * 1e3, 3),
            "bit_exact_and_parity_vs_oracle": bool(ok),
            "encode_note": "spec_encode_tree: generated size passes bottom-up, record scan, generated writers table "
                           "by table top-down (each row its own bytes, children placed into gaps); HIP events, no host sync"}


def e2e_decode(stream_host, ends_host, dev, reps=5, chunks=8):
    """Pinned host -> H2D -> decode -> D2H of all columns + status, pipelined in record chunks
    over three streams (spec_amd.HostDecoder); whole-pipeline rate (Mmsg/s)."""
    n = ends_host.numel()
    hd = spec_amd.HostDecoder(FLAT16, n, stream_host.numel(), dev, chunks=chunks)
    hd.decode(stream_host, ends_host)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        hd.decode(stream_host, ends_host)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    return n / dt / 1e6, dt, hd


def main(argv=None):
    args = parse(argv)
    env = spec_env()
    if env and not args.allow_env:
        sys.exit(f"bench.py: SPEC_AMD_* variables set ({', '.join(env)}); unset them or pass --allow-env")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        launch_ranks(args, argv if argv is not None else sys.argv[1:])
        return
    global _RESULT_OUT
    # the collective libraries print to fd 1 (gloo: "[Gloo] Rank k is connected ...", RCCL its
    # version banner at the first communicator): send everything but the result line to stderr,
    # so stdout carries exactly one JSON line
    sys.stdout.flush()
    _RESULT_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    run(args, env)


def run(args, env):
    dist, rank, world, dev = dist_setup(args)
    devices = distinct_devices(dist, dev)
    n = args.records
    cols, heaps, d_cols, d_heaps, stream, ends = make_batch(n, args.seed + rank, dev)
    stream_bytes = stream.numel()
    mean_rec = stream_bytes / n

    if args.no_jit:
        spec_amd.set_jit(False)
    jit = spec_amd.lib().spec_decode_flat_prepare(FLAT16.c, stream_bytes, n) == 1
    dec = spec_amd.Decoder(FLAT16, stream, ends)
    out_cols, status = dec.cols, dec.status
    gpu_prewarm(dec)
    elapsed = time_decode(dec, args.steps, args.warmup, dist)
    elapsed = max_over_ranks(dist, elapsed)
    total_records = sum_over_ranks(dist, float(n)) * args.steps
    value = total_records / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    # per-launch kernel time on the launch stream (HIP events)
    avg_ms, med_ms, p10_ms, p90_ms = kernel_time_events(dec, max(20, args.steps), spread=True)
    alg_bytes = stream_bytes + n * (8 + COLUMN_BYTES + 1)
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9
    read_only = (stream_bytes + 8 * n) / (avg_ms * 1e-3) / 1e9

    # HBM bytes per launch from the committed rocprofv3 PMC passes (tools/pmc_traffic.py):
    # FETCH_SIZE x 2 (gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE, for this kernel
    # The passes record the device-source revision they measured (source_rev): a traffic figure
    # measured on other kernel code is not reported (traffic null, traffic_rev says which).
    traffic, traffic_rev = None, None
    kname = "spec_decode_flat_pair_jit" if jit else "decode_flat_kernel"
    rev = source_rev()
    if os.path.exists(args.traffic):
        try:
            t = json.load(open(args.traffic)).get(kname, {})
            traffic_rev = t.get("source_rev")
            if t.get("records") == n and traffic_rev == rev:
                traffic = t.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    torch.cuda.synchronize()
    checks = {"status_all_ok": int((status != 0).sum().item()) == 0}
    extras = {}
    if not args.no_verify:
        extras["verify"] = verify_sample(cols, heaps, stream, ends, out_cols, status, VERIFY_RECORDS)
        checks.update({k: v for k, v in extras["verify"].items() if k != "records"})
    if not args.no_extras:
        enc = spec_amd.Encoder(FLAT16, n, dev)
        out = torch.empty(stream_bytes, dtype=torch.uint8, device=dev)
        e2 = torch.empty(n, dtype=torch.int64, device=dev)
        enc_ms, _ = kernel_time_events(lambda: enc.encode_into(d_cols, d_heaps, out, e2), 10)
        torch.cuda.synchronize()
        enc_same = torch.equal(out, stream) and torch.equal(e2, ends)
        checks["encode_repeat_bit_exact"] = bool(enc_same)
        heap_bytes = sum(h.numel() for h in d_heaps.values())
        enc_alg = n * (COLUMN_BYTES + 8) + heap_bytes + stream_bytes
        extras["encode"] = {"mmsg_s": round(n / (enc_ms * 1e-3) / 1e6, 1),
                            "gb_s": round(enc_alg / (enc_ms * 1e-3) / 1e9, 1),
                            "frac": round(enc_alg / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "alg_bytes": int(enc_alg),
                            "ms": round(enc_ms, 4), "bit_exact_vs_decode_input": bool(enc_same)}
        if rank == 0 and world == 1 and not args.no_cpu:
            try:
                extras["encode"]["cpu_baseline"] = cpu_encode_baseline(cols, heaps, n, stream_bytes, args.cpu_seconds)
            except Exception as e:
                extras["encode"]["cpu_baseline"] = {"error": repr(e)[:300]}
        if not args.no_jit and jit:
            try:
                extras["decode_generic"] = generic_leg(stream, ends, out_cols, status, avg_ms)
                checks["generic_same_columns"] = extras["decode_generic"]["same_columns"]
            except Exception as e:  # an extra leg never hides the headline line
                extras["decode_generic"] = {"error": repr(e)[:300]}
        try:
            extras["decode_errmask"] = errmask_leg(stream, ends, out_cols, status, avg_ms)
            checks["errmask_same_columns"] = extras["decode_errmask"]["same_columns"]
        except Exception as e:
            extras["decode_errmask"] = {"error": repr(e)[:300]}
        if args.shard_total > 0:
            try:
                extras["config5_sharded"] = shard_leg(args, dist, rank, world, dev)
            except Exception as e:
                extras["config5_sharded"] = {"error": repr(e)[:300]}
        if rank == 0:  # one-GPU legs: at N>1 rank 0 runs them on its own device after the timed region
            try:
                extras["decode_wide"] = wide_leg(dev)
                checks["wide_parity"] = all(v["jit_vs_generic_same"] and v["oracle_sample_ok"]
                                            for v in extras["decode_wide"].values())
            except Exception as e:
                extras["decode_wide"] = {"error": repr(e)[:300]}
            try:
                extras["nested"] = nested_leg(n, args.seed, dev,
                                              0.0 if (args.no_cpu or world > 1) else args.cpu_seconds)
            except Exception as e:
                extras["nested"] = {"error": repr(e)[:300]}
            try:
                extras["tree_pkg1"] = tree_leg(dev)
                checks["tree_parity"] = extras["tree_pkg1"]["bit_exact_and_parity_vs_oracle"]
            except Exception as e:
                extras["tree_pkg1"] = {"error": repr(e)[:300]}
        if rank == 0:
            try:
                sh = stream.cpu().pin_memory()
                eh = ends.cpu().pin_memory()
                rate, dt, hd = e2e_decode(sh, eh, dev)
                hcols, hst = hd.columns()
                e2e_ok = bool(torch.equal(hst, status.cpu()) and torch.equal(hcols[13], out_cols[13].cpu())
                              and torch.equal(hcols[0], out_cols[0].cpu()))
                extras["e2e_pinned_decode"] = {
                    "mmsg_s": round(rate, 1), "ms": round(dt * 1e3, 3), "ok": e2e_ok,
                    "note": f"pinned H2D stream+ends, decode, D2H columns+status; {hd.chunks} record chunks "
                            "pipelined over 3 streams, one D2H per chunk (chunk-major outputs)",
                    "pcie_bytes": int(sh.numel() + 8 * n + n * (COLUMN_BYTES + 1))}
            except Exception as e:
                extras["e2e_pinned_decode"] = {"error": repr(e)[:300]}
            try:
                extras["frames_index"] = frames_leg(stream, ends, dev)
            except Exception as e:
                extras["frames_index"] = {"error": repr(e)[:300]}
            try:
                extras["lz4"] = lz4_leg(stream, ends, dev)
            except Exception as e:
                extras["lz4"] = {"error": repr(e)[:300]}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        s_np = stream.cpu().numpy()
        e_np = ends.cpu().numpy().view(np.uint64)
        res, threads, sample = cpu_baseline(s_np, e_np, args.cpu_seconds)
        cpu = {"value": round(res[threads], 2), "unit": "Mmsg/s", "cores": threads, "kind": "port",
               "sample": f"{sample} Flat16 records (the full batch) decoded repeatedly for ~{args.cpu_seconds/2:.0f} s "
                         f"per thread count on {threads} host threads (all cores this process may use) and on 1; "
                         f"C restatement of OpenMessageErr + 16 getters",
               "single_core_value": round(res[1], 2), "host_model": host_cpu_model()}

    # the native one-process multi-device leg (spec_shard_*): a child of rank 0 drives every device
    # while the ranks wait (the others on the rendezvous store: no GPU work of theirs runs meanwhile)
    if not args.no_native and not args.no_extras:
        if rank == 0:
            extras["native_shard"] = native_leg_isolated(args, world, devices)
            if "columns_ok" in extras["native_shard"]:
                checks["native_shard_columns"] = extras["native_shard"]["columns_ok"]
        if dist is not None:
            import datetime

            store = dist.distributed_c10d._get_default_store()
            if rank == 0:
                store.set("spec_native_done", "1")
            else:
                store.wait(["spec_native_done"], datetime.timedelta(minutes=15))

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mmsg/s",
            "n_gpus": devices,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": "flat16-decode", "records_per_gpu": n,
                       "mean_record_bytes": round(mean_rec, 1), "stream_bytes_per_gpu": stream_bytes,
                       "parallelism": f"record-sharded x{world}, no collective",
                       "ranks": world, "distinct_devices": devices,
                       "rehearsal": devices < world,
                       "backend": args.backend if world > 1 else None, "env": env},
            "gb_s": round(total_records * (mean_rec + 8 + COLUMN_BYTES + 1) / elapsed / 1e9, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": kname, "kernel_ms_avg": round(avg_ms, 5),
                         "kernel_ms_median": round(med_ms, 5), "kernel_ms_p10": round(p10_ms, 5),
                         "kernel_ms_p90": round(p90_ms, 5), "alg_bytes_per_launch": alg_bytes,
                         "read_only_gb_s": round(read_only, 1), "source_rev": rev, "traffic_rev": traffic_rev},
            "cpu_baseline": cpu,
            "correct": bool(all(checks.values())),
            "checks": checks,
        }
        line.update(extras)
        print(json.dumps(line), file=_RESULT_OUT or sys.stdout, flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
