"""The native multi-device path (include/spec_amd.h spec_shard_*, spec_amd.shard.NativeShard):
one process, one stream + RCCL communicator per visible device, a host batch split into
contiguous shards, every shard decoded on its device into a packed buffer, one gather to the
root device — against the oracle's decode of the whole batch (spans rebased by the shards'
byte bases).  On a one-GPU box the flow runs with one device (the gather is the root's own
copy); with more devices the gather goes through RCCL send/recv."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from spec_amd import FLAT16, workload
from spec_amd.shard import NativeShard, PackedColumns
from tests.test_shard_gloo import rebase_spans

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 4099, 300_001])
def test_native_shard_decode_gather(dev, n):
    ndev = torch.cuda.device_count()
    sh = NativeShard(list(range(ndev)))
    cols, heaps = workload.flat16(n, seed=n % 97)
    stream, ends = O.encode_flat_batch(FLAT16.tags, FLAT16.kinds, cols, [heaps.get(f) for f in range(16)], n)
    packs, bases = sh.decode_host(FLAT16, stream, ends)
    gathered = sh.gather(packs, root=0)
    sh.sync()
    want, wst = O.decode_flat_batch(FLAT16.tags, FLAT16.kinds, stream, ends, FLAT16.widths, 8)
    g = gathered.cpu()
    views, off = [], 0
    for k in range(ndev):
        r0, r1 = sh.bounds(n, k)
        nb = PackedColumns.nbytes_for(FLAT16, r1 - r0)
        views.append(PackedColumns(FLAT16, r1 - r0, "cpu", buf=g[off: off + nb]))
        off += nb
        assert bases[k] == (int(ends[r0 - 1]) if r0 else 0)
    for f, fld in enumerate(FLAT16.fields):
        got = rebase_spans([v.cols[f] for v in views], bases, fld.kind.name in ("STRING", "BYTES"))
        assert np.array_equal(got, want[f]), fld
    assert np.array_equal(np.concatenate([v.status.numpy() for v in views]), wst)


def test_native_shard_rejects_duplicate_devices():
    from spec_amd import SpecError

    with pytest.raises(SpecError):
        NativeShard([0, 0])
