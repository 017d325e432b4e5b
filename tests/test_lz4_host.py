"""spec_lz4_frame_blocks (host walk of LZ4 frame headers / block size words, C ABI) against the
oracle's frame layout: the blocks it lists decompress (oracle) to the frame's content, an open
frame is carried across calls, corrupt headers and capacity are reported."""
import numpy as np

import spec_amd
from oracle import oracle as O
from spec_amd.lz4 import Lz4State, frame_blocks


def content_of(buf, blocks, block_max):
    out = []
    for b in blocks:
        raw = buf[int(b["src_off"]):int(b["src_off"]) + int(b["src_len"])].tobytes()
        out.append(raw if b["stored"] else O.lz4_decompress_block(raw, block_max))
    return b"".join(out)


def test_blocks_of_frames():
    rng = np.random.default_rng(1)
    data = np.concatenate([rng.integers(0, 4, 500000, dtype=np.uint8), rng.integers(0, 256, 80000, dtype=np.uint8)])
    for bcs in (False, True):
        f = O.lz4_frame_write(data, [1000, 300000, data.size], 256 << 10, block_checksum=bcs)
        blocks, used, bmax, rc = frame_blocks(f)
        assert rc == 0 and used == f.size and bmax == 256 << 10
        assert any(b["stored"] for b in blocks)  # the random tail is stored uncompressed
        assert content_of(f, blocks, bmax) == data.tobytes()
    # two frames back to back + a skippable frame between them
    f1 = O.lz4_frame_write(data[:1000], None, 64 << 10)
    f2 = O.lz4_frame_write(data[1000:5000], None, 64 << 10)
    skip = np.frombuffer(b"\x50\x2a\x4d\x18" + (3).to_bytes(4, "little") + b"xyz", np.uint8)
    buf = np.concatenate([f1, skip, f2])
    blocks, used, bmax, rc = frame_blocks(buf)
    assert rc == 0 and used == buf.size and content_of(buf, blocks, bmax) == data[:5000].tobytes()


def test_open_frame_across_calls():
    """A live connection: the frame never closes, bytes arrive in arbitrary pieces."""
    rng = np.random.default_rng(2)
    data = rng.integers(0, 3, 900000, dtype=np.uint8)
    f = O.lz4_frame_write(data, [10000, 400000, data.size], 256 << 10, close=False)
    st = Lz4State()
    got, pos = b"", 0
    for cut in (5, 6, 100, 70000, 200000, 500000, f.size):
        piece = f[pos:cut]
        blocks, used, bmax, rc = frame_blocks(piece, st)
        assert rc == 0
        got += content_of(piece, blocks, 256 << 10)
        pos += used
    assert got == data.tobytes() and st.in_frame == 1


def test_corrupt_and_capacity():
    data = np.arange(200000, dtype=np.uint32).view(np.uint8)
    f = O.lz4_frame_write(data, None, 64 << 10)
    g = f.copy()
    g[6] ^= 0xFF  # header checksum
    assert frame_blocks(g)[3] == -6
    g = f.copy()
    g[0] = 0  # magic
    assert frame_blocks(g)[3] == -6
    blocks, used, _, rc = frame_blocks(f, cap=2)
    assert rc == -4 and len(blocks) == 2 and used == int(blocks[1]["src_off"] + blocks[1]["src_len"])
    assert frame_blocks(f[:3])[1:] == (0, 0, 0)


def test_content_checksum_reported():
    """The frame's stored content checksum (xxh32 of its content, what lz4.Reader verifies at the
    end mark) is reported in the state of the call that reaches the end mark, and only there."""
    rng = np.random.default_rng(4)
    data = rng.integers(0, 8, 300_000, dtype=np.uint8)
    f = O.lz4_frame_write(data, [100_000, data.size], 64 << 10)
    st = Lz4State()
    blocks, used, _, rc = frame_blocks(f[: f.size // 2], st)
    assert rc == 0 and not (st.flags & 4) and st.in_frame
    blocks, used2, _, rc = frame_blocks(f[used:], st)
    assert rc == 0 and (st.flags & 4) and not st.in_frame
    assert st.content_checksum == O.xxh32(data)
    # no content checksum in the frame: bit 2 stays clear
    g = O.lz4_frame_write(data, None, 64 << 10, content_checksum=False)
    st2 = Lz4State()
    frame_blocks(g, st2)
    assert not (st2.flags & 4) and st2.content_checksum == 0
