"""Field-level errors (spec_decode_flat_errors): per record, which getters' *Err variants
(internal/types/msg.go:233-459) return an error, against the oracle's *Err getters — values
written as one kind and read as another (range and type errors), extremes, fuzzed records.
Every test runs under the schema-specialised kernel's errmask variant (hiprtc) and the
precompiled generic kernel."""
from __future__ import annotations

import numpy as np
import pytest

from oracle import oracle as O
from spec_amd import FLAT16, Schema, workload
from tests.gpu_helpers import check_errors, concat_records, oracle_encode
from tests.test_gpu_flat import ALL_KINDS, _extreme_values, write_record

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["jit", "generic"])
def kernel(request):
    import spec_amd

    spec_amd.set_jit(request.param == "jit")
    yield request.param
    spec_amd.set_jit(True)


@pytest.mark.parametrize("shift", [0, 1, 2, 3, 5, 8, 13])
def test_cross_kind_errors(dev, shift):
    rng = np.random.default_rng(shift)
    m = 48
    per_kind = {k: _extreme_values(k, rng, m) for k in ALL_KINDS}
    recs = [write_record([(t + 1, k, per_kind[k][i]) for t, k in enumerate(ALL_KINDS)]) for i in range(m)]
    stream, ends = concat_records(recs)
    read = Schema([(t + 1, ALL_KINDS[(t + shift) % len(ALL_KINDS)]) for t in range(len(ALL_KINDS))])
    mask = check_errors(dev, read, stream, ends, f"shift={shift}")
    if shift:
        assert mask.any()  # some getters err (type mismatches)


def test_flat16_no_errors(dev):
    cols, heaps = workload.flat16(5000, seed=4)
    stream, ends = oracle_encode(FLAT16, cols, heaps, 5000)
    assert not check_errors(dev, FLAT16, stream, ends, "flat16").any()


@pytest.mark.parametrize("seed", range(3))
def test_fuzz_errors(dev, seed):
    rng = np.random.default_rng(50 + seed)
    n = 3000
    cols, heaps = workload.flat16(n, seed=seed)
    stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    s = stream.copy()
    idx = rng.integers(0, s.size, s.size // 100)
    s[idx] = rng.integers(0, 256, idx.size, dtype=np.uint8)
    check_errors(dev, FLAT16, s, ends, f"fuzz {seed}")


def test_fast_path_errors(dev):
    """Natural-type records (the specialised kernel's fast path accepts them) whose decoders
    still err: float32 +-Inf (the MaxFloat32 range check, internal/decode/float.go:15-32),
    malformed varints and string lengths past the record start."""
    n = 4000
    cols, heaps = workload.flat16(n, seed=8)
    f32 = cols[8].view(np.uint32).reshape(-1).copy()
    f32[::7] = 0x7F800000  # +Inf
    f32[3::11] = 0xFF800000  # -Inf
    f32[5::13] = 0x7FC00001  # NaN passes
    cols[8] = f32.view(np.uint8).reshape(n, 4)
    stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    s = stream.copy()
    rng = np.random.default_rng(3)
    for i in rng.integers(0, n, 200):  # corrupt a byte just below some record's table
        s[int(ends[i]) - 52 - int(rng.integers(0, 6))] ^= 0x80
    mask = check_errors(dev, FLAT16, s, ends, "fast path errors")
    assert (mask & (1 << 8)).any()
