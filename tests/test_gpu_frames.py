"""GPU frame index (spec_frames_index_device) against the oracle's restatement of the mpx read
loop (oracle.frames_read, mpx/conn_reader.go:179-194) and, where the test builds the frames
from known message sizes, against the cumulative sum of those sizes: the same ends, count,
consumed and capacity status, on mpx frame buffers of every shape the parallel algorithm
distinguishes (segment boundaries, incomplete tails, frames longer than the entry window ->
serial fallback, tiny frames -> step cap -> fallback, garbage, buffers only 4-byte aligned)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import spec_amd
from oracle import oracle as O
from spec_amd import FLAT16, workload
from tests.gpu_helpers import to_dev

pytestmark = pytest.mark.gpu

SEG = 32768  # frames_device.hip FI_SEG


def frames_of(sizes, rng, tail=b""):
    out = bytearray()
    for z in sizes:
        out += int(z).to_bytes(4, "big")
        out += rng.integers(0, 256, int(z), dtype=np.uint8).tobytes()
    return np.frombuffer(bytes(out) + tail, dtype=np.uint8)


def check(dev, buf, cap=None, label="", sizes=None, offset=0):
    """Device index of buf (placed `offset` bytes into a 256-byte aligned allocation) vs the
    oracle read loop; with `sizes`, also vs cumsum(4 + size) of the frames the test wrote."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    cap_h = cap if cap is not None else max(1, buf.size // 4)
    want_ends, want_used = O.frames_read(buf, cap_h)
    over = want_ends is None
    if over:  # more than cap complete frames: the first cap of them
        want_ends, _ = O.frames_read(buf, buf.size // 4 + 1)
        want_ends = want_ends[:cap_h]
        want_used = int(want_ends[-1]) if cap_h else 0
    if sizes is not None:
        known = np.cumsum(np.asarray(sizes, np.uint64) + np.uint64(4))
        k = want_ends.size
        assert np.array_equal(known[:k], want_ends), f"{label}: oracle vs known sizes"
    room = torch.zeros(offset + max(buf.size, 4), dtype=torch.uint8)
    room[offset: offset + buf.size] = torch.from_numpy(buf)
    d = room.to(dev)[offset: offset + buf.size]
    ends, used, st = spec_amd.frames_index_device(d, cap_h)
    got = ends.cpu().numpy().view(np.uint64)
    assert used == want_used, f"{label}: consumed {used} vs {want_used}"
    assert np.array_equal(got, want_ends), f"{label}: ends differ ({got.size} vs {want_ends.size} frames)"
    assert st == (-4 if over else 0), f"{label}: status {st}"
    # the host indexer (product, CPU) agrees too
    h_ends, h_used = spec_amd.frames_index(buf, cap_h)
    assert np.array_equal(h_ends, want_ends) and h_used == want_used, f"{label}: host walk"


@pytest.mark.parametrize("seed", range(3))
def test_random_frames(dev, seed):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, 600, 20000)
    check(dev, frames_of(sizes, rng), label=f"random {seed}", sizes=sizes)
    check(dev, frames_of(sizes, rng), label=f"random {seed} at +4", sizes=sizes, offset=4)
    # incomplete tails: a partial head, a partial frame
    check(dev, frames_of(sizes[:5000], rng, tail=b"\x00\x00"), label="partial head")
    check(dev, frames_of(sizes[:5000], rng, tail=b"\x00\x00\x01\x00" + b"x" * 100), label="partial frame")


def test_segment_boundaries(dev):
    """Frames ending exactly on 32 KiB segment boundaries, heads straddling them, a stream that ends
    exactly at a boundary."""
    rng = np.random.default_rng(9)
    for first in (SEG - 4, SEG - 5, SEG - 6, SEG - 7, SEG - 2048 - 4, SEG - 2049 - 4):
        sizes = [first] + list(rng.integers(0, 300, 500))
        check(dev, frames_of(sizes, rng), label=f"first={first}", sizes=sizes)
        check(dev, frames_of(sizes, rng), label=f"first={first} at +12", sizes=sizes, offset=12)
    sizes = [SEG - 4] * 3
    check(dev, frames_of(sizes, rng), label="exact segments", sizes=sizes)


def test_sub_segment_windows(dev):
    """The 4 KiB sub-segment tables inside a segment: frames 1-2 KiB long (heads past a
    sub-segment's 1024-byte window, so the walk runs on into the next sub-segment), 4 KiB frames
    landing exactly on sub-segment starts, heads at window offsets WS - 1 / WS, and frames so
    small that a segment has more live entries than the emit's records."""
    rng = np.random.default_rng(11)
    sub, ws = 4096, 512  # frames_device.hip FI_SUB, FI_WS
    cases = {
        "1-2 KiB": list(rng.integers(1000, 2000, 600)),
        "3-4 KiB": list(rng.integers(3000, 4000, 300)),
        "exact sub": [sub - 4] * 40,
        "window 1023": [sub + ws - 1 - 4] + list(rng.integers(0, 300, 2000)),
        "window 1024": [sub + ws - 4] + list(rng.integers(0, 300, 2000)),
        "mixed": list(rng.choice([7, 60, 900, 1100, 1500, 2040, 4092], 3000)),
        # ~70 true heads in a segment's 2048-byte entry window: more live entries than the 32
        # records kept, so some segments' emits rebuild their tables (the work list)
        "small": list(rng.integers(6, 36, 30000)),
    }
    for label, sizes in cases.items():
        check(dev, frames_of(sizes, rng), label=label, sizes=sizes)
        check(dev, frames_of(sizes, rng), label=f"{label} at +20", sizes=sizes, offset=20)


def test_long_frames_fall_back(dev):
    """Frames longer than the 2048-byte entry window (and > 64 KiB) take the serial walk."""
    rng = np.random.default_rng(4)
    sizes = list(rng.integers(0, 300, 2000)) + [5000, 70000, 3] + list(rng.integers(0, 300, 2000))
    check(dev, frames_of(sizes, rng), label="long frames", sizes=sizes)


def test_tiny_frames_fall_back(dev):
    """Empty messages (4-byte frames): > 4096 frames per segment -> step cap -> serial walk."""
    check(dev, np.zeros(4 * 70000, np.uint8), label="empty frames")


def test_capacity_and_small(dev):
    rng = np.random.default_rng(2)
    buf = frames_of(rng.integers(0, 100, 3000), rng)
    for cap in (1, 10, 2999, 3000, 3001):
        check(dev, buf, cap=cap, label=f"cap {cap}")
        check(dev, buf, cap=cap, label=f"cap {cap} at +4", offset=4)
    for n in (0, 1, 3, 4):
        check(dev, np.zeros(n, np.uint8) + 0, label=f"len {n}")
    check(dev, np.array([0, 0, 0, 1, 7], np.uint8), label="one byte frame")


def test_garbage(dev):
    rng = np.random.default_rng(8)
    for k in range(3):
        buf = rng.integers(0, 256, 200000, dtype=np.uint8)
        buf[::97] = 0
        check(dev, buf, label=f"garbage {k}")


def test_flat16_frames_then_decode(dev):
    """The receive path on the device: frames indexed on the GPU, decoded in place."""
    n = 100_000
    cols, heaps = workload.flat16(n, seed=6)
    stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
    frames = spec_amd.make_frames(stream, ends)
    d = to_dev(frames, dev)
    fends, used, st = spec_amd.frames_index_device(d, n)
    assert st == 0 and used == frames.size and fends.numel() == n
    got = spec_amd.decode_frames(FLAT16, d, fends)
    want = spec_amd.decode_flat(FLAT16, to_dev(stream, dev), to_dev(ends.view(np.int64), dev))
    torch.cuda.synchronize()
    assert torch.equal(got.status, want.status)
    for f in range(16):
        if FLAT16.kinds[f] in (spec_amd.Kind.STRING, spec_amd.Kind.BYTES):
            continue  # spans are relative to different buffers
        assert torch.equal(got.cols[f], want.cols[f]), f
