"""The HIP path against the committed golden fixtures (tests/golden/*.npz) — fixed bytes, no
oracle in the loop: decode of the fixture stream gives the fixture columns, encode of the
fixture columns gives the fixture stream."""
from __future__ import annotations

import os

import numpy as np
import pytest

import spec_amd
from spec_amd import FLAT16, NESTED
from tests.gpu_helpers import to_dev

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(params=["jit", "generic"])
def kernel(request):
    spec_amd.set_jit(request.param == "jit")
    yield request.param
    spec_amd.set_jit(True)


def test_flat16_golden(dev, kernel):
    import torch

    g = np.load(os.path.join(GOLDEN, "flat16_small.npz"), allow_pickle=False)
    n = len(g["ends"])
    got = spec_amd.decode_flat(FLAT16, to_dev(g["stream"], dev), to_dev(g["ends"].view(np.int64), dev))
    torch.cuda.synchronize()
    assert np.array_equal(got.status.cpu().numpy(), g["status"])
    for f in range(16):
        assert np.array_equal(got.cols[f].cpu().numpy(), g[f"dec{f}"]), f
    cols = [to_dev(g[f"col{f}"], dev) for f in range(16)]
    heaps = {f: to_dev(g[f"heap{f}"], dev) for f in range(16) if f"heap{f}" in g}
    out, ends = spec_amd.encode_flat(FLAT16, cols, heaps, n)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), g["stream"])
    assert np.array_equal(ends.cpu().numpy().view(np.uint64), g["ends"])


def test_nested_golden_roundtrip(dev):
    import torch

    g = np.load(os.path.join(GOLDEN, "nested_small.npz"), allow_pickle=False)
    n = len(g["ends"])
    w = {k[3:]: g[k] for k in g.files if k.startswith("in_")}
    m = len(w["key"])
    outer = [to_dev(w["id"], dev), to_dev(w["seq"].view(np.uint8).reshape(n, 8), dev),
             to_dev(w["name"].view(np.uint8).reshape(n, 8), dev), None]
    items = [to_dev(w["key"].view(np.uint8).reshape(m, 4), dev), to_dev(w["value"].view(np.uint8).reshape(m, 8), dev),
             to_dev(w["label"].view(np.uint8).reshape(m, 8), dev)]
    out, ends = spec_amd.encode_nested(NESTED, outer, {2: to_dev(w["name_heap"], dev)},
                                       to_dev(w["item_begin"].view(np.int32), dev), items,
                                       {2: to_dev(w["label_heap"], dev)}, n)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), g["stream"])
    d = spec_amd.decode_nested(NESTED, to_dev(g["stream"], dev), to_dev(g["ends"].view(np.int64), dev))
    torch.cuda.synchronize()
    assert np.array_equal(d.item_begin.cpu().numpy().view(np.uint32), g["out_item_begin"])
    assert np.array_equal(d.items[0].cpu().numpy().view(np.int32).ravel(), g["out_key"])
    assert np.array_equal(d.outer[0].cpu().numpy(), g["out_id"])
