"""GPU parity for spec_parse_messages (recursive ParseMessage validation)
against the oracle on the same inputs."""
from __future__ import annotations

import numpy as np
import pytest

import spec_amd
from oracle import oracle as O
from spec_amd import FLAT16, workload
from tests.gpu_helpers import concat_records, oracle_encode, to_dev
from tests.test_oracle_parse import _msg, _raw_message

pytestmark = pytest.mark.gpu


def check_parse(dev, stream, ends, head=0, label=""):
    import torch

    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    want_st, want_sz = O.parse_batch(stream, ends, head)
    d_stream = to_dev(stream if stream.size else np.zeros(1, np.uint8), dev)[: stream.size]
    st, sz = spec_amd.parse_messages(d_stream, to_dev(ends.view(np.int64), dev), head)
    torch.cuda.synchronize()
    gst, gsz = st.cpu().numpy(), sz.cpu().numpy().view(np.uint32)
    if not np.array_equal(gst, want_st):
        i = int(np.nonzero(gst != want_st)[0][0])
        raise AssertionError(f"{label}: record {i}: gpu={gst[i]} oracle={want_st[i]}")
    assert np.array_equal(gsz, want_sz), label
    return gst


def test_parse_flat16_and_nested(dev):
    n = 5000
    cols, heaps = workload.flat16(n, seed=21)
    stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    st = check_parse(dev, stream, ends, label="flat16")
    assert not st.any()
    w = workload.nested(n, seed=22)
    s2, e2 = O.encode_nested_batch(w)
    st = check_parse(dev, s2, e2, label="nested")
    assert not st.any()


def test_parse_classes(dev):
    good = _msg([(1, "int64", 5), (2, "string", "abc")])
    inf32 = O.encode("float32", float("inf"))[0]
    lst_items = O.encode("int64", 1)[0] + O.encode("int64", 2)[0]
    swapped = lst_items + O.encode_list_table(len(lst_items), [4, 2])[0]
    recs = [good, b"", bytes([0xFF, 80]), _raw_message([inf32]), _raw_message([bytes([1, 2, 3, 99])]),
            _raw_message([swapped]), _raw_message([good]), _raw_message([O.encode("struct", 3)[0]])]
    stream, ends = concat_records(recs * 40)
    check_parse(dev, stream, ends, label="classes")


def test_parse_nesting_depth(dev):
    """Messages nested 20 deep parse; beyond 32 containers the engine reports TOO_DEEP
    (the reference recurses without a bound: documented limit)."""
    import torch

    def nest(d):
        b = _msg([(1, "int32", 7)])
        for _ in range(d):
            b = _raw_message([b])
        return b

    stream, ends = concat_records([nest(20)] * 70)
    check_parse(dev, stream, ends, label="depth 20")
    stream, ends = concat_records([nest(40)] * 3)
    st, _ = spec_amd.parse_messages(to_dev(stream, dev), to_dev(ends.view(np.int64), dev))
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 8).all()


@pytest.mark.parametrize("seed", range(4))
def test_parse_fuzz(dev, seed):
    rng = np.random.default_rng(900 + seed)
    n = 3000
    if seed % 2:
        stream, ends = O.encode_nested_batch(workload.nested(n, seed=seed))
    else:
        cols, heaps = workload.flat16(n, seed=seed)
        stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    recs = [bytes(stream[(int(ends[i - 1]) if i else 0):int(ends[i])]) for i in range(n)]
    out = []
    for r in recs:
        b = bytearray(r)
        x = rng.integers(0, 4)
        if x == 0:
            for _ in range(rng.integers(1, 4)):
                b[rng.integers(0, len(b))] = rng.integers(0, 256)
        elif x == 1:
            b = b[:rng.integers(0, len(b))]
        elif x == 2:
            b = b[rng.integers(0, len(b)):]
        out.append(bytes(b))
    s2, e2 = concat_records(out)
    check_parse(dev, s2, e2, label=f"fuzz {seed}")


def test_parse_frames(dev):
    n = 1000
    cols, heaps = workload.flat16(n, seed=5)
    stream, ends = oracle_encode(FLAT16, cols, heaps, n)
    fr = spec_amd.make_frames(stream, ends)
    fends, _ = spec_amd.frames_index(fr)
    check_parse(dev, fr, fends, head=4, label="frames")
