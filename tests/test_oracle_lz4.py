"""The LZ4 oracle (oracle/lz4.c: mpx's compression, pierrec/lz4/v4 restated from the published
formats).  pierrec is absent, so the exact compressed bytes are parity-unpinned; what is pinned
here: xxHash32 known answers, hand-made blocks (literal-only, overlapping matches, the error
classes of pierrec's decodeBlock), and round trips of the compressor/decompressor and of the
frame writer/reader (header checksum, block/content checksums, stored blocks, flushes)."""
import numpy as np

from oracle import oracle as O


def test_xxh32_known_answers():
    # XXH32 reference values (xxHash specification test vectors)
    assert O.xxh32(b"") == 0x02CC5D05
    assert O.xxh32(b"", 1) == 0x0B2CB792


def test_hand_made_blocks():
    # literal-only block: token 0x50, "hello"
    assert O.lz4_decompress_block(b"\x50hello", 100) == b"hello"
    # "ab" then a match of 6 at offset 2 (overlapping copy repeats the pattern), then 1 literal
    blk = bytes([0x22]) + b"ab" + bytes([2, 0]) + bytes([0x10]) + b"z"
    assert O.lz4_decompress_block(blk, 100) == b"ab" + b"abababab"[:6] + b"z"
    # run-length: 1 literal, offset 1, match 4 + 15 + 10 = 29
    blk = bytes([0x1F]) + b"x" + bytes([1, 0, 10])
    assert O.lz4_decompress_block(blk, 100) == b"x" * 30
    # long literal run: 15 + 255 + 5 = 275 bytes
    lit = bytes(range(256)) + bytes(19)
    blk = bytes([0xF0, 255, 5]) + lit
    assert O.lz4_decompress_block(blk, 1000) == lit
    # error classes: empty, offset 0, offset beyond the output start, a match nibble with no
    # offset, literal overrun, output overrun
    assert O.lz4_decompress_block(b"", 10) is None
    assert O.lz4_decompress_block(bytes([0x10]) + b"a" + bytes([0, 0]), 10) is None
    assert O.lz4_decompress_block(bytes([0x10]) + b"a" + bytes([2, 0]), 10) is None
    assert O.lz4_decompress_block(bytes([0x11]) + b"a", 10) is None
    assert O.lz4_decompress_block(bytes([0x50]) + b"abc", 10) is None
    assert O.lz4_decompress_block(b"\x50hello", 4) is None


def test_block_round_trips():
    rng = np.random.default_rng(3)
    for data in [b"", b"a", b"abcd" * 1000, rng.integers(0, 256, 5000, dtype=np.uint8).tobytes(),
                 (b"spec message " * 50 + rng.integers(0, 4, 300, dtype=np.uint8).tobytes()) * 40]:
        c = O.lz4_compress_block(data)
        assert O.lz4_decompress_block(c, len(data)) == data
    # compressible data shrinks
    assert len(O.lz4_compress_block(b"abcd" * 1000)) < 200


def test_frame_round_trips():
    rng = np.random.default_rng(5)
    data = np.concatenate([rng.integers(0, 8, 300000, dtype=np.uint8),
                           rng.integers(0, 256, 100000, dtype=np.uint8)])
    for bcs in (False, True):
        for flushes in ([data.size], [1000, 70000, 262144 + 5, data.size]):
            f = O.lz4_frame_write(data, flushes, 256 << 10, content_checksum=True, block_checksum=bcs)
            assert f[:4].tobytes() == b"\x04\x22\x4d\x18"
            rc, out, used = O.lz4_frame_read(f, data.size + 10)
            assert rc == 0 and used == f.size and np.array_equal(out, data)
    # header checksum, content checksum, corrupt block
    f = O.lz4_frame_write(data, None, 64 << 10)
    g = f.copy()
    g[6] ^= 1
    assert O.lz4_frame_read(g, data.size)[0] == -2
    g = f.copy()
    g[-1] ^= 1
    assert O.lz4_frame_read(g, data.size)[0] == -6
    # an unclosed frame (a live connection): every complete block, the partial one left
    f = O.lz4_frame_write(data, [200000, data.size], 64 << 10, close=False)
    rc, out, used = O.lz4_frame_read(f[:-100], data.size)
    assert rc == 0 and used < f.size - 100 and np.array_equal(out, data[:out.size]) and out.size % 1 == 0
