"""GPU LZ4 decompression (spec_lz4_decompress + spec_lz4_pack) against the oracle (oracle/lz4.c):
every block of oracle-written frames decompressed on the device equals the content; corrupt
blocks get the oracle's verdict; short and long literals, near / far / overlapping matches and
sequences too long for the batch window are all exercised; and the whole compressed receive path (LZ4 frame -> blocks -> device
decompress -> device frame index -> in-place decode) equals the oracle decode."""
from __future__ import annotations

import numpy as np
import pytest

import spec_amd
from oracle import oracle as O
from spec_amd import FLAT16, workload
from spec_amd.lz4 import decompress, frame_blocks
from tests.gpu_helpers import to_dev

pytestmark = pytest.mark.gpu


def gpu_content(dev, f):
    blocks, used, bmax, rc = frame_blocks(f)
    assert rc == 0
    out, sizes, status = decompress(to_dev(f, dev), blocks, bmax)
    return out.cpu().numpy(), status.cpu().numpy()


def _chunks(rng, n, lit, rep):
    """random runs of `lit` bytes, each followed by `rep` bytes copied from earlier output"""
    out = bytearray()
    while len(out) < n:
        out += rng.integers(0, 256, lit, dtype=np.uint8).tobytes()
        src = int(rng.integers(0, max(1, len(out) - rep)))
        out += out[src:src + rep]
    return np.frombuffer(bytes(out[:n]), np.uint8)


@pytest.mark.parametrize("kind", ["text", "random", "mixed", "zeros", "period3", "period200", "records", "chunks",
                                  "longlit"])
def test_frames_round_trip(dev, kind):
    rng = np.random.default_rng(hash(kind) % 1000)
    n = 700000
    data = {
        "text": np.frombuffer((b"spec message field table trailer " * 30000)[:n], np.uint8),
        "random": rng.integers(0, 256, n, dtype=np.uint8),
        "mixed": np.concatenate([rng.integers(0, 6, n // 2, dtype=np.uint8), rng.integers(0, 256, n - n // 2,
                                                                                           dtype=np.uint8)]),
        "zeros": np.zeros(n, np.uint8),          # one match per block far longer than the ring
        "period3": np.frombuffer((b"abc" * n)[:n], np.uint8),
        "period200": np.tile(rng.integers(0, 256, 200, dtype=np.uint8), n // 200 + 1)[:n],
        # many short sequences, near and far matches, batch windows filling up
        "records": np.tile(np.frombuffer(b"".join(bytes([7, i % 13, 0, 0]) + rng.integers(0, 256, 9, dtype=np.uint8)
                                                  .tobytes() for i in range(64)), np.uint8), n // 832 + 1)[:n],
        "chunks": _chunks(rng, n, 300, 700),  # literals > 16 bytes, matches reaching back up to a block
        "longlit": _chunks(rng, n, 9000, 3000),  # literals longer than the ring look-ahead: alone, HBM to HBM
    }[kind]
    for flushes in ([n], [1, 4000, 300001, n]):
        f = O.lz4_frame_write(data, flushes, 256 << 10)
        got, st = gpu_content(dev, f)
        assert not st.any()
        assert np.array_equal(got, data), kind


def test_block_sizes(dev):
    rng = np.random.default_rng(4)
    for bmax in (64 << 10, 1 << 20):
        data = rng.integers(0, 10, 3_000_000, dtype=np.uint8)
        f = O.lz4_frame_write(data, None, bmax)
        got, st = gpu_content(dev, f)
        assert np.array_equal(got, data)


def test_corrupt_blocks(dev):
    """Hand-made blocks: the device status equals the oracle's verdict block by block."""
    import torch

    good = O.lz4_compress_block(b"hello hello hello hello hello!")
    cases = [good, b"\x50hello", b"", bytes([0x10]) + b"a" + bytes([0, 0]), bytes([0x10]) + b"a" + bytes([2, 0]),
             bytes([0x11]) + b"a", bytes([0x50]) + b"abc", bytes([0xF0]), bytes([0x1F]) + b"x" + bytes([1, 0, 10]),
             bytes([0x0F, 1, 0])]
    src = b"".join(cases)
    blocks = np.zeros(len(cases), spec_amd.lz4.BLOCK_DTYPE)
    off = 0
    for i, c in enumerate(cases):
        blocks[i] = (off, len(c), 0)
        off += len(c)
    d = to_dev(np.frombuffer(src + b"\0\0\0\0", np.uint8), dev)[: len(src)]
    L = spec_amd.lib()
    import ctypes as C
    nb, slot = len(cases), 1024
    d_blocks = to_dev(blocks.view(np.uint8), dev)
    slots = torch.zeros(nb * slot, dtype=torch.uint8, device=dev)
    sizes = torch.zeros(nb, dtype=torch.int32, device=dev)
    status = torch.zeros(nb, dtype=torch.uint8, device=dev)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    assert L.spec_lz4_decompress(p(d), len(src), p(d_blocks), nb, p(slots), slot, p(sizes), p(status), None) == 0
    torch.cuda.synchronize()
    st, sz, sl = status.cpu().numpy(), sizes.cpu().numpy().view(np.uint32), slots.cpu().numpy()
    for i, c in enumerate(cases):
        want = O.lz4_decompress_block(c, slot)
        assert bool(st[i]) == (want is None), (i, c)
        if want is not None:
            assert sz[i] == len(want) and sl[i * slot:i * slot + len(want)].tobytes() == want, i


def test_compressed_receive_path(dev):
    """mpx with compression: Flat16 records -> frames -> one LZ4 frame (flushed per ~500 frames)
    -> host block walk -> device decompress -> device frame index -> in-place decode."""
    import torch

    n = 50_000
    cols, heaps = workload.flat16(n, seed=12)
    stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
    frames = spec_amd.make_frames(stream, ends)
    fe = spec_amd.frames_index(frames, n)[0]
    flushes = list(fe[499::500]) + [frames.size]
    comp = O.lz4_frame_write(frames, flushes, 256 << 10, close=False)
    blocks, used, bmax, rc = frame_blocks(comp)
    assert rc == 0 and used == comp.size
    plain, sizes, status = decompress(to_dev(comp, dev), blocks, bmax)
    assert plain.numel() == frames.size
    fends, consumed, st = spec_amd.frames_index_device(plain, n)
    assert st == 0 and consumed == frames.size and fends.numel() == n
    got = spec_amd.decode_frames(FLAT16, plain, fends)
    want_cols, want_status = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, stream, ends, FLAT16.widths, nthreads=4)
    torch.cuda.synchronize()
    assert np.array_equal(got.status.cpu().numpy(), want_status)
    for f in range(16):
        if FLAT16.kinds[f] in (spec_amd.Kind.STRING, spec_amd.Kind.BYTES):
            continue  # spans point into the framed buffer, not the compact stream
        assert np.array_equal(got.cols[f].cpu().numpy(), want_cols[f]), f


@pytest.mark.parametrize("chunks", [[0], [5], [16], [17, 3, 40], [1000, 1, 15, 16, 4096, 77777], [300_000]])
def test_content_checksum_device(dev, chunks):
    """spec_lz4_content_update / _digest: xxHash32 streamed over any split of the data (empty,
    partial stripes carried between calls, long runs), equal to the oracle's xxh32."""
    import torch

    from spec_amd.lz4 import ContentChecksum

    rng = np.random.default_rng(sum(chunks))
    data = rng.integers(0, 256, sum(chunks), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev) if data.size else torch.zeros(0, dtype=torch.uint8, device=dev)
    cc = ContentChecksum(dev)
    p = 0
    for c in chunks:
        cc.update(d[p: p + c])
        p += c
    assert cc.digest() == O.xxh32(data)


def test_content_checksum_receive_path(dev):
    """A compressed connection's frame end: the blocks decompressed on the device, the content
    checksum computed on the device over the decompressed bytes equals the one the frame stores
    (frame_blocks reports it), and a corrupted stored checksum is detected."""
    import torch

    from spec_amd.lz4 import ContentChecksum, Lz4State

    n = 20_000
    cols, heaps = workload.flat16(n, seed=8)
    stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
    fr = spec_amd.make_frames(stream, ends)
    comp = O.lz4_frame_write(fr, None, 256 << 10)
    st = Lz4State()
    blocks, used, bmax, rc = frame_blocks(comp, st)
    assert rc == 0 and (st.flags & 4)
    out, _, _ = decompress(torch.from_numpy(comp).to(dev), blocks, bmax)
    cc = ContentChecksum(dev)
    cc.update(out)
    assert cc.digest() == st.content_checksum == O.xxh32(fr)
    bad = comp.copy()
    bad[-1] ^= 0x40  # the stored checksum's last byte
    st2 = Lz4State()
    frame_blocks(bad, st2)
    assert (st2.flags & 4) and st2.content_checksum != cc.digest()
