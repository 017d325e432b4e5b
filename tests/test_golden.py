"""The oracle against the committed golden fixtures (tests/golden/, made by make_golden.py).

The fixtures are oracle-generated (the reference holds no byte vectors):
this pins the oracle against drift, and the same files drive tests/test_gpu_golden.py."""
from __future__ import annotations

import os

import numpy as np

from oracle import oracle as O
from spec_amd import workload
from spec_amd.schema import FLAT16

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def test_flat16_golden_encode():
    g = load("flat16_small.npz")
    n = len(g["ends"])
    cols = [g[f"col{f}"] for f in range(16)]
    heaps = [g[f"heap{f}"] if f"heap{f}" in g else None for f in range(16)]
    stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, heaps, n)
    assert np.array_equal(stream, g["stream"])
    assert np.array_equal(ends, g["ends"])


def test_flat16_golden_decode():
    g = load("flat16_small.npz")
    dec, status = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, g["stream"], g["ends"], FLAT16.widths)
    assert np.array_equal(status, g["status"]) and not status.any()
    for f in range(16):
        assert np.array_equal(dec[f], g[f"dec{f}"]), f


def test_flat16_golden_roundtrip_values():
    """decode(encode(cols)) == cols for every fixed-width field; spans address the same bytes."""
    g = load("flat16_small.npz")
    s = g["stream"]
    for f, fld in enumerate(FLAT16.fields):
        if fld.width and f"heap{f}" not in g:
            assert np.array_equal(g[f"dec{f}"], g[f"col{f}"]), fld
        else:
            d, c, h = g[f"dec{f}"].view(np.uint32), g[f"col{f}"].view(np.uint32), g[f"heap{f}"]
            for i in range(len(d)):
                assert bytes(s[d[i, 0]:d[i, 0] + d[i, 1]]) == bytes(h[c[i, 0]:c[i, 0] + c[i, 1]])


def test_flat16_workload_is_deterministic():
    g = load("flat16_small.npz")
    cols, heaps = workload.flat16(len(g["ends"]))
    for f in range(16):
        assert np.array_equal(cols[f], g[f"col{f}"])


def test_flat16_mean_record_size():
    """the benchmark records average 256 +- 4 B."""
    n = 20000
    cols, heaps = workload.flat16(n, seed=1)
    stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
    assert 250 <= len(stream) / n <= 260


def test_nested_golden():
    g = load("nested_small.npz")
    w = {k[3:]: g[k] for k in g.files if k.startswith("in_")}
    stream, ends = O.encode_nested_batch(w)
    assert np.array_equal(stream, g["stream"]) and np.array_equal(ends, g["ends"])
    d = O.decode_nested_batch(stream, ends)
    for k, v in d.items():
        assert np.array_equal(v, g[f"out_{k}"]), k
    assert np.array_equal(d["counts"], np.diff(w["item_begin"]))
    assert np.array_equal(d["key"], w["key"])
    assert np.array_equal(d["value"].view(np.uint64), w["value"].view(np.uint64))
    assert np.array_equal(d["id"], w["id"]) and np.array_equal(d["seq"], w["seq"])
