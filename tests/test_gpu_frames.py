"""GPU frame index (spec_frames_index_device) against the host walk (spec_frames_index): the
same ends, count, consumed and capacity status, on mpx frame buffers of every shape the
parallel algorithm distinguishes (segment boundaries, incomplete tails, frames longer than the
entry window -> serial fallback, tiny frames -> step cap -> fallback, garbage)."""
from __future__ import annotations

import numpy as np
import pytest

import spec_amd
from oracle import oracle as O
from spec_amd import FLAT16, workload
from tests.gpu_helpers import to_dev

pytestmark = pytest.mark.gpu

SEG = 65536


def frames_of(sizes, rng, tail=b""):
    out = bytearray()
    for z in sizes:
        out += int(z).to_bytes(4, "big")
        out += rng.integers(0, 256, int(z), dtype=np.uint8).tobytes()
    return np.frombuffer(bytes(out) + tail, dtype=np.uint8)


def check(dev, buf, cap=None, label=""):
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    cap_h = cap if cap is not None else max(1, buf.size // 4)
    want_ends, want_used = spec_amd.frames_index(buf, cap_h)
    d = to_dev(buf if buf.size else np.zeros(4, np.uint8), dev)[: buf.size]
    ends, used, st = spec_amd.frames_index_device(d, cap_h)
    got = ends.cpu().numpy().view(np.uint64)
    assert used == want_used, f"{label}: consumed {used} vs {want_used}"
    assert np.array_equal(got, want_ends), f"{label}: ends differ ({got.size} vs {want_ends.size} frames)"
    # capacity status as the host call's return code
    more = spec_amd.frames_index(buf, max(1, buf.size // 4 + 1))[0].size
    assert st == (-4 if more > cap_h else 0), f"{label}: status {st}"


@pytest.mark.parametrize("seed", range(3))
def test_random_frames(dev, seed):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, 600, 20000)
    check(dev, frames_of(sizes, rng), label=f"random {seed}")
    # incomplete tails: a partial head, a partial frame
    check(dev, frames_of(sizes[:5000], rng, tail=b"\x00\x00"), label="partial head")
    check(dev, frames_of(sizes[:5000], rng, tail=b"\x00\x00\x01\x00" + b"x" * 100), label="partial frame")


def test_segment_boundaries(dev):
    """Frames ending exactly on 64 KiB boundaries, heads straddling them, a stream that ends
    exactly at a boundary."""
    rng = np.random.default_rng(9)
    for first in (SEG - 4, SEG - 5, SEG - 6, SEG - 7, SEG - 2048 - 4, SEG - 2049 - 4):
        sizes = [first] + list(rng.integers(0, 300, 500))
        check(dev, frames_of(sizes, rng), label=f"first={first}")
    sizes = [SEG - 4] * 3
    check(dev, frames_of(sizes, rng), label="exact segments")


def test_long_frames_fall_back(dev):
    """Frames longer than the 2048-byte entry window (and > 64 KiB) take the serial walk."""
    rng = np.random.default_rng(4)
    sizes = list(rng.integers(0, 300, 2000)) + [5000, 70000, 3] + list(rng.integers(0, 300, 2000))
    check(dev, frames_of(sizes, rng), label="long frames")


def test_tiny_frames_fall_back(dev):
    """Empty messages (4-byte frames): > 4096 frames per segment -> step cap -> serial walk."""
    check(dev, np.zeros(4 * 70000, np.uint8), label="empty frames")


def test_capacity_and_small(dev):
    rng = np.random.default_rng(2)
    buf = frames_of(rng.integers(0, 100, 3000), rng)
    for cap in (1, 10, 2999, 3000, 3001):
        check(dev, buf, cap=cap, label=f"cap {cap}")
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
    import torch

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
