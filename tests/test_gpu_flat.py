"""GPU parity: the HIP decode/encode path (through include/spec_amd.h) against the CPU oracle
on the same inputs, bit for bit.  Edge cases follow what the reference's tests exercise
(internal/decode/*_test.go, internal/writer/*_test.go) plus malformed-input fuzzing."""
from __future__ import annotations

import struct

import numpy as np
import pytest

import spec_amd
from oracle import oracle as O
from spec_amd import Field, Kind, Schema, workload
from tests.gpu_helpers import check_decode, check_encode, concat_records, oracle_encode

pytestmark = pytest.mark.gpu

FLAT16 = spec_amd.FLAT16

ALL_KINDS = [Kind(k) for k in range(1, 16)]  # the flat column kinds
ORACLE_NAME = {
    Kind.BOOL: "bool", Kind.BYTE: "byte", Kind.INT16: "int16", Kind.INT32: "int32",
    Kind.INT64: "int64", Kind.UINT16: "uint16", Kind.UINT32: "uint32", Kind.UINT64: "uint64",
    Kind.FLOAT32: "float32", Kind.FLOAT64: "float64", Kind.BIN64: "bin64",
    Kind.BIN128: "bin128", Kind.BIN256: "bin256", Kind.STRING: "string", Kind.BYTES: "bytes",
}


def write_record(fields):
    """fields: [(tag, Kind, value)] written in order with the oracle Writer -> bytes"""
    w = O.Writer()
    w.message()
    for tag, kind, v in fields:
        err = w.field(tag, ORACLE_NAME[kind], v)
        assert err is None, err
    data, err = w.end()
    assert err is None, err
    w.close()
    return data


@pytest.fixture(params=["jit", "generic"])
def kernel(request):
    """Run a test with the schema-specialised kernels (hiprtc) and with the generic kernel."""
    spec_amd.set_jit(request.param == "jit")
    yield request.param
    spec_amd.set_jit(True)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4096 + 17])
def test_flat16_decode_parity(dev, kernel, n):
    cols, heaps = workload.flat16(n, seed=n)
    stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    check_decode(dev, FLAT16, stream, ends, f"flat16 n={n}")


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4096 + 17])
def test_flat16_encode_bitexact(dev, kernel, n):
    cols, heaps = workload.flat16(n, seed=n + 1)
    check_encode(dev, FLAT16, cols, heaps, n, f"flat16 n={n}")


def test_flat16_full_size_parity(dev, kernel):
    """BASELINE configs 2+3 at full size: 1M Flat16 records, encode bit-exact and decode
    identical to the oracle."""
    n = 1 << 20
    cols, heaps = workload.flat16(n)
    stream, ends = check_encode(dev, FLAT16, cols, heaps, n, "flat16 1M encode")
    check_decode(dev, FLAT16, stream, ends, "flat16 1M decode")


def test_roundtrip_property(dev):
    """decode(encode(columns)) == columns; string/bytes spans point at the same payload."""
    import torch

    n = 50_000
    cols, heaps = workload.flat16(n, seed=99)
    d_cols = [torch.from_numpy(c).to(dev) for c in cols]
    d_heaps = {f: torch.from_numpy(h).to(dev) for f, h in heaps.items()}
    out, ends = spec_amd.encode_flat(FLAT16, d_cols, d_heaps, n)
    got = spec_amd.decode_flat(FLAT16, out, ends)
    assert int((got.status != 0).sum()) == 0
    s = out.cpu().numpy()
    for f, fld in enumerate(FLAT16.fields):
        g = got.cols[f].cpu().numpy()
        if fld.kind in (Kind.STRING, Kind.BYTES):
            gs, ws = g.view(np.uint32), cols[f].view(np.uint32)
            assert np.array_equal(gs[:, 1], ws[:, 1])
            for i in range(0, n, 997):
                a = s[gs[i, 0]:gs[i, 0] + gs[i, 1]]
                b = heaps[f][ws[i, 0]:ws[i, 0] + ws[i, 1]]
                assert np.array_equal(a, b)
        else:
            assert np.array_equal(g, cols[f]), fld


def _extreme_values(kind, rng, m):
    if kind == Kind.BOOL:
        return [True, False] * (m // 2)
    if kind == Kind.BYTE:
        return [0, 255, 1, 128] * (m // 4)
    ints = {
        Kind.INT16: [0, 1, -1, 32767, -32768, 63, -64, 64],
        Kind.INT32: [0, 1, -1, 2**31 - 1, -2**31, 32767, 32768, -32769],
        Kind.INT64: [0, 1, -1, 2**63 - 1, -2**63, 2**31, -2**31 - 1, 32768],
        Kind.UINT16: [0, 1, 65535, 127, 128, 255, 256, 16384],
        Kind.UINT32: [0, 1, 2**32 - 1, 65535, 65536, 2**28, 127, 128],
        Kind.UINT64: [0, 1, 2**64 - 1, 2**32 - 1, 2**32, 65536, 2**63, 127],
    }
    if kind in ints:
        vals = ints[kind]
        return [vals[i % len(vals)] for i in range(m)]
    if kind == Kind.FLOAT32:
        bits = [0, 0x80000000, 0x7F800000, 0xFF800000, 0x7FC00001, 0x7F800123, 0x00000001,
                0x007FFFFF, 0x7F7FFFFF, 0x3F800000]
        return [struct.unpack("<f", struct.pack("<I", bits[i % len(bits)]))[0] for i in range(m)]
    if kind == Kind.FLOAT64:
        bits = [0, 0x8000000000000000, 0x7FF0000000000000, 0x7FF0000000000001, 0x7FF8000000000123,
                0x47EFFFFFE0000000, 0x47EFFFFFE0000001, 0x47EFFFFFF0000000, 0x36A0000000000000,
                0x3690000000000000, 0x3690000000000001, 0x380FFFFFF0000000, 0x0000000000000001,
                0xC7EFFFFFE0000000, 0x3FF0000000000001, 0x3FF0000010000000]
        return [struct.unpack("<d", struct.pack("<Q", bits[i % len(bits)]))[0] for i in range(m)]
    if kind in (Kind.BIN64, Kind.BIN128, Kind.BIN256):
        w = {Kind.BIN64: 8, Kind.BIN128: 16, Kind.BIN256: 32}[kind]
        return [rng.integers(0, 256, w, dtype=np.uint8).tobytes() for _ in range(m)]
    if kind == Kind.STRING:
        return ["", "a", "hello, world"] * (m // 3) + ["x" * 200] * (m - 3 * (m // 3))
    if kind == Kind.BYTES:
        return [b"", b"\x00", b"\xff" * 9] * (m // 3) + [b"z" * 300] * (m - 3 * (m // 3))
    raise ValueError(kind)


@pytest.mark.parametrize("shift", range(1, len(ALL_KINDS)))
def test_cross_kind_decode(dev, kernel, shift):
    """Values written as kind A, read back with the getter of kind B: the cross-width and
    range-check rules of internal/decode/{int,uint,float}.go, type mismatches => zero."""
    rng = np.random.default_rng(shift)
    m = 48
    per_kind = {k: _extreme_values(k, rng, m) for k in ALL_KINDS}
    recs = []
    for i in range(m):
        recs.append(write_record([(t + 1, k, per_kind[k][i]) for t, k in enumerate(ALL_KINDS)]))
    stream, ends = concat_records(recs)
    read = Schema([(t + 1, ALL_KINDS[(t + shift) % len(ALL_KINDS)]) for t in range(len(ALL_KINDS))])
    check_decode(dev, read, stream, ends, f"cross-kind shift={shift}")


def test_same_kind_extremes(dev, kernel):
    rng = np.random.default_rng(5)
    m = 80
    per_kind = {k: _extreme_values(k, rng, m) for k in ALL_KINDS}
    recs = [write_record([(t + 1, k, per_kind[k][i]) for t, k in enumerate(ALL_KINDS)]) for i in range(m)]
    stream, ends = concat_records(recs)
    schema = Schema([(t + 1, k) for t, k in enumerate(ALL_KINDS)])
    check_decode(dev, schema, stream, ends, "extremes")


def test_float_widths_both_ways(dev, kernel):
    """float32 <-> float64 through the getters (float.go:15-78): NaN payloads, Inf, subnormal
    rounding, the MaxFloat32 boundary."""
    rng = np.random.default_rng(11)
    recs = []
    f32 = _extreme_values(Kind.FLOAT32, rng, 40)
    f64 = _extreme_values(Kind.FLOAT64, rng, 48)
    rnd = rng.integers(0, 2**63, 200, dtype=np.uint64)
    f64 += [struct.unpack("<d", struct.pack("<Q", int(b)))[0] for b in rnd]
    for i in range(len(f64)):
        recs.append(write_record([(1, Kind.FLOAT32, f32[i % len(f32)]), (2, Kind.FLOAT64, f64[i])]))
    stream, ends = concat_records(recs)
    for schema in (Schema([(1, Kind.FLOAT64), (2, Kind.FLOAT32)]), Schema([(1, Kind.FLOAT32), (2, Kind.FLOAT64)])):
        check_decode(dev, schema, stream, ends, "float widths")


def test_empty_and_zero_records(dev, kernel):
    recs = [b"", write_record([]), b"", write_record([(1, Kind.BOOL, True)]), b""]
    stream, ends = concat_records(recs)
    check_decode(dev, FLAT16, stream, ends, "empty records")
    stream, ends = concat_records([b""] * 130)
    check_decode(dev, FLAT16, stream, ends, "all empty")


def test_handcrafted_tables(dev, kernel):
    """Unsorted, duplicate, missing and extra tags; end offsets beyond dataSize; big-format
    tables with small values; truncated trailers (msg_test.go:74-143 error classes)."""
    vals = [O.encode("int32", 7)[0], O.encode("string", "abc")[0], O.encode("int64", -5)[0],
            O.encode("bool", True)[0], O.encode("uint16", 300)[0]]
    data = b"".join(vals)
    ends_in_data = list(np.cumsum([len(v) for v in vals]))
    recs = []
    tag_sets = [
        [4, 14, 5, 1, 6],          # unsorted
        [4, 4, 5, 5, 6],           # duplicates
        [1, 2, 3, 4, 5],           # wrong tags for the values
        [4, 14, 16, 20, 200],      # sorted, extra tags
        [2, 4, 6, 8, 10],
        [16, 15, 14, 5, 4],        # reversed
        [1, 1, 1, 1, 1],
    ]
    for tags in tag_sets:
        fields = list(zip(tags, [int(e) for e in ends_in_data]))
        trailer, _, err = O.encode_message_table(len(data), fields)
        assert err is None
        recs.append(data + trailer)
        # end offsets past dataSize
        bad = [(t, int(e) + 1000) for t, e in fields]
        recs.append(data + O.encode_message_table(len(data), bad)[0])
        # big table (tag > 255 forces the 6-byte format)
        big = fields + [(300, int(ends_in_data[-1]))]
        recs.append(data + O.encode_message_table(len(data), big)[0])
    # error classes from internal/decode/msg_test.go
    recs.append(bytes([0xFF, 80]))                                        # invalid table size
    recs.append(bytes([0xFF]) + O.put_reverse_uint32(1000) + bytes([80]))  # invalid data size
    recs.append(bytes([0, 0, 80, 0]) + O.put_reverse_uint32(1000) + bytes([80]))  # invalid table
    recs.append(bytes([0, 0, 80]) + O.put_reverse_uint32(1000) + bytes([0, 80]))  # invalid data
    recs.append(data + bytes([70]))                                       # invalid type
    recs.append(bytes([3, 0, 80]))                                        # table size % 3 != 0
    stream, ends = concat_records(recs)
    schema = Schema([(4, Kind.INT32), (14, Kind.STRING), (5, Kind.INT64), (1, Kind.BOOL),
                     (6, Kind.UINT16), (16, Kind.INT64), (300, Kind.UINT16)])
    check_decode(dev, schema, stream, ends, "handcrafted")
    check_decode(dev, FLAT16, stream, ends, "handcrafted/flat16")


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_mutated_records(dev, kernel, seed):
    """Valid Flat16 records with random byte mutations, truncations and garbage records."""
    rng = np.random.default_rng(1000 + seed)
    n = 3000
    cols, heaps = workload.flat16(n, seed=seed)
    stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    recs = [bytes(stream[(int(ends[i - 1]) if i else 0):int(ends[i])]) for i in range(n)]
    out = []
    for r in recs:
        x = rng.integers(0, 6)
        b = bytearray(r)
        if x == 0:
            for _ in range(rng.integers(1, 4)):
                b[rng.integers(0, len(b))] = rng.integers(0, 256)
        elif x == 1:  # mutate the trailer / table region
            for _ in range(rng.integers(1, 3)):
                b[len(b) - 1 - rng.integers(0, min(len(b), 60))] = rng.integers(0, 256)
        elif x == 2:
            b = b[rng.integers(0, len(b)):]
        elif x == 3:
            b = b[:rng.integers(0, len(b))]
        elif x == 4:
            b = bytearray(rng.integers(0, 256, rng.integers(0, 300), dtype=np.uint8).tobytes())
            if len(b) and rng.integers(0, 2):
                b[-1] = 80
        out.append(bytes(b))
    s2, e2 = concat_records(out)
    check_decode(dev, FLAT16, s2, e2, f"fuzz seed={seed}")


COMPACT_SCHEMAS = [
    [(1, Kind.INT32), (2, Kind.FLOAT64), (3, Kind.STRING)],              # the NESTED item schema
    [(1, Kind.BOOL), (2, Kind.INT64), (3, Kind.STRING), (4, Kind.FLOAT64)],
    [(7, Kind.UINT16)],
    [(5, Kind.INT32), (9, Kind.BYTES)],
]


@pytest.mark.parametrize("si", range(len(COMPACT_SCHEMAS)))
def test_fuzz_compact_records(dev, kernel, si):
    """Schemas of <= 4 fields, whose trailer and table sit in one 16-byte tail window (the
    decoder's compact fast path): data sizes with 1-, 2- and 3-byte varints, mutated
    trailers/tables, truncations, garbage — against the oracle."""
    rng = np.random.default_rng(77 + si)
    fields = COMPACT_SCHEMAS[si]
    n = 1500
    lens = [0, 3, 100, 200, 20000]
    recs = []
    for i in range(n):
        vals = []
        for tag, kind in fields:
            if kind == Kind.INT32:
                v = int(rng.integers(-2**31, 2**31))
            elif kind == Kind.INT64:
                v = int(rng.integers(-2**63, 2**63, dtype=np.int64))
            elif kind == Kind.UINT16:
                v = int(rng.integers(0, 2**16))
            elif kind == Kind.BOOL:
                v = bool(rng.integers(0, 2))
            elif kind == Kind.FLOAT64:
                v = float(rng.standard_normal())
            elif kind == Kind.STRING:
                v = "s" * lens[int(rng.integers(0, len(lens) - (0 if i % 50 == 0 else 1)))]
            else:
                v = bytes(rng.integers(0, 256, lens[int(rng.integers(0, 4))], dtype=np.uint8))
            vals.append((tag, kind, v))
        b = bytearray(write_record(vals))
        x = rng.integers(0, 6)
        if x == 0:
            b[len(b) - 1 - rng.integers(0, min(len(b), 16))] = rng.integers(0, 256)
        elif x == 1:
            b = b[:rng.integers(0, len(b))]
        elif x == 2:
            b = bytearray(rng.integers(0, 256, rng.integers(0, 40), dtype=np.uint8).tobytes())
            if len(b) > 2:
                b[-1], b[-2] = 80, 3 * len(fields)
        recs.append(bytes(b))
    stream, ends = concat_records(recs)
    check_decode(dev, Schema(fields), stream, ends, f"compact schema {si}")


def test_large_records_global_path(dev, kernel):
    """Records too large for a wave's LDS slab take the direct-HBM path; big messages
    (dataSize > 65535) use the 6-byte table."""
    rng = np.random.default_rng(3)
    recs = []
    for i in range(200):
        ln = int(rng.choice([10, 500, 3000, 70000]))
        recs.append(write_record([(1, Kind.INT64, i - 100), (2, Kind.STRING, "s" * ln),
                                  (3, Kind.BYTES, bytes(rng.integers(0, 256, ln // 3, dtype=np.uint8))),
                                  (4, Kind.FLOAT64, 1.5 * i)]))
    stream, ends = concat_records(recs)
    schema = Schema([(1, Kind.INT64), (2, Kind.STRING), (3, Kind.BYTES), (4, Kind.FLOAT64)])
    check_decode(dev, schema, stream, ends, "large records")


def _cols_for(schema, n, seed, str_len=(30, 62)):
    return workload.gen_columns(schema, n, seed, str_len=str_len)


@pytest.mark.parametrize("case", ["all_kinds", "unsorted_tags", "dup_tags", "big_tags", "long_strings",
                                  "empty_strings", "single", "no_fields"])
def test_encode_schemas(dev, kernel, case):
    n = 777
    if case == "all_kinds":
        schema = Schema([(t + 1, k) for t, k in enumerate(ALL_KINDS)])
        sl = (0, 40)
    elif case == "unsorted_tags":
        schema = Schema([(9, Kind.INT64), (3, Kind.STRING), (200, Kind.BOOL), (1, Kind.UINT32), (50, Kind.BIN128)])
        sl = (30, 62)
    elif case == "dup_tags":
        schema = Schema([(5, Kind.INT32), (2, Kind.INT64), (5, Kind.STRING), (2, Kind.BYTE), (5, Kind.FLOAT64)])
        sl = (30, 62)
    elif case == "big_tags":
        schema = Schema([(1, Kind.INT32), (256, Kind.STRING), (70000 % 65536, Kind.UINT64)])
        sl = (30, 62)
    elif case == "long_strings":
        schema = Schema([(1, Kind.STRING), (2, Kind.INT16), (3, Kind.BYTES)])
        sl = (20000, 40000)
        n = 70
    elif case == "empty_strings":
        schema = Schema([(1, Kind.STRING), (2, Kind.BYTES)])
        sl = (0, 0)
    elif case == "single":
        schema = Schema([(7, Kind.UINT64)])
        sl = (0, 0)
    else:
        schema = Schema([])
        sl = (0, 0)
    cols, heaps = _cols_for(schema, n, 17, sl)
    stream, ends = check_encode(dev, schema, cols, heaps, n, case)
    check_decode(dev, schema, stream, ends, case + "/decode")


@pytest.mark.parametrize("n", [1000, 4096 + 33])
def test_encode_pair_groups_over_slab(dev, kernel, n):
    """64-record groups whose bytes exceed the write pass's slab (long strings: written straight
    to HBM) among groups staged in LDS, single long records inside staged groups, a partial last
    block and group — the bytes stay the oracle Writer's.  (It was written for the wave-pair write
    pass, encode_write_pair_body, built with -DSPEC_AB_ENC_PAIR=1, and passed there too.)"""
    a_cols, a_heaps = workload.flat16(n, seed=21)
    b_cols, b_heaps = workload.gen_columns(FLAT16, n, 22, str_len=(300, 700))
    big = np.zeros(n, bool)
    for g in (2, 9, (n - 1) // 64):
        big[64 * g: 64 * g + 64] = True
    big[5::97] = True  # single long records inside staged groups
    cols = [np.where(big[:, None], b, a) for a, b in zip(a_cols, b_cols)]
    heaps = {}
    for f, h in a_heaps.items():
        heaps[f] = np.concatenate([h, b_heaps[f]])
        sp = cols[f].view(np.uint32).reshape(n, 2).copy()
        sp[big, 0] += h.size  # b's spans index the second part of the joined heap
        cols[f] = sp.view(np.uint8).reshape(n, 8)
    check_encode(dev, FLAT16, cols, heaps, n, f"flat16 pair groups n={n}")


def test_encode_capacity_and_errors(dev, kernel):
    import torch

    schema = Schema([(1, Kind.STRING)])
    n = 100
    cols, heaps = _cols_for(schema, n, 1)
    d_cols = [torch.from_numpy(c).to(dev) for c in cols]
    d_heap = torch.from_numpy(heaps[0]).to(dev)
    enc = spec_amd.Encoder(schema, n, dev)
    total = int(enc.size(d_cols).item())
    out = torch.zeros(total - 1, dtype=torch.uint8, device=dev)
    ends = torch.zeros(n, dtype=torch.int64, device=dev)
    enc.encode_into(d_cols, {0: d_heap}, out, ends)
    torch.cuda.synchronize()
    assert int(enc.total.item()) == total  # reports the required size
    assert int(out.abs().sum()) == 0 and int(ends.abs().sum()) == 0  # nothing written
    # a span outside its heap is an encoder error
    bad = cols[0].copy()
    bad.view(np.uint32)[5, 0] = heaps[0].size
    with pytest.raises(spec_amd.SpecError):
        spec_amd.encode_flat(schema, [torch.from_numpy(bad).to(dev)], {0: d_heap}, n)


def test_zero_records(dev):
    import torch

    s = torch.zeros(0, dtype=torch.uint8, device=dev)
    e = torch.zeros(0, dtype=torch.int64, device=dev)
    got = spec_amd.decode_flat(FLAT16, s, e)
    assert got.status.numel() == 0


def test_decode_range_and_host_pipeline(dev):
    """spec_decode_flat_range over chunks == one full decode; the pinned-host pipeline
    (HostDecoder: chunked H2D / decode / D2H on three streams) returns the same columns."""
    import ctypes as C

    import torch

    n = 70_001
    cols, heaps = workload.flat16(n, seed=4)
    stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, stream, ends, FLAT16.widths, nthreads=4)
    d_stream = torch.from_numpy(stream).to(dev)
    d_ends = torch.from_numpy(ends.view(np.int64)).to(dev)
    out = spec_amd.alloc_columns(FLAT16, n, dev)
    st = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    ptrs = (C.c_void_p * 16)(*[c.data_ptr() for c in out])
    L = spec_amd.lib()
    for r0, r1 in [(0, 1000), (1000, 1001), (1001, 33333), (33333, n)]:
        b0 = int(ends[r0 - 1]) if r0 else 0
        rc = L.spec_decode_flat_range(C.byref(FLAT16.c), C.c_void_p(d_stream.data_ptr()), stream.size,
                                      C.c_void_p(d_ends.data_ptr()), r0, r1, int(ends[r1 - 1]) - b0, ptrs,
                                      C.c_void_p(st.data_ptr()), None)
        assert rc == 0
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), wst)
    for f in range(16):
        assert np.array_equal(out[f].cpu().numpy(), want[f]), f
    h_stream = torch.from_numpy(stream).pin_memory()
    h_ends = torch.from_numpy(ends.view(np.int64)).pin_memory()
    for chunks in (5, 16):
        hd = spec_amd.HostDecoder(FLAT16, n, stream.size, dev, chunks=chunks)
        hd.decode(h_stream, h_ends)
        hcols, hst = hd.columns()
        assert np.array_equal(hst.numpy(), wst), chunks
        for f in range(16):
            assert np.array_equal(hcols[f].numpy(), want[f]), (chunks, f)
        r0, r1, c3, s3 = hd.chunk(3)
        assert np.array_equal(c3[13].numpy(), want[13][r0:r1]) and np.array_equal(s3.numpy(), wst[r0:r1])


def test_decode_frames_in_place(dev, kernel):
    """mpx frames decoded in place == the same records decoded from a compact stream (spans
    shifted by the 4-byte heads before them)."""
    import torch

    n = 3001
    cols, heaps = workload.flat16(n, seed=12)
    stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, stream, ends, FLAT16.widths, nthreads=4)
    fr = spec_amd.make_frames(stream, ends)
    fends, used = spec_amd.frames_index(fr)
    assert used == fr.size
    got = spec_amd.decode_frames(FLAT16, torch.from_numpy(fr).to(dev), torch.from_numpy(fends.view(np.int64)).to(dev))
    torch.cuda.synchronize()
    assert np.array_equal(got.status.cpu().numpy(), wst)
    shift = 4 * (np.arange(n, dtype=np.uint32) + 1)
    for f, fld in enumerate(FLAT16.fields):
        g = got.cols[f].cpu().numpy()
        w = want[f].copy()
        if fld.kind in (Kind.STRING, Kind.BYTES):
            wv = w.view(np.uint32)
            wv[:, 0] = np.where(wv[:, 1] > 0, wv[:, 0] + shift, 0)
        assert np.array_equal(g, w), fld
