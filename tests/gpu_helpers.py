"""Shared helpers for the GPU parity tests: run the HIP path through the C ABI and the CPU
oracle on the same inputs and compare bit for bit."""
from __future__ import annotations

import numpy as np
import torch

import spec_amd
from oracle import oracle as O


def oracle_encode(schema, cols, heaps, n):
    return O.encode_flat_batch(schema.tags, schema.kinds, cols, [heaps.get(f) for f in range(len(schema))], n)


def to_dev(a: np.ndarray, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def check_decode(dev, schema, stream: np.ndarray, ends: np.ndarray, label=""):
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    want_cols, want_status = O.decode_flat_batch(schema.tags, schema.kinds, stream, ends, schema.widths,
                                                 nthreads=4)
    d_stream = to_dev(stream if stream.size else np.zeros(1, np.uint8), dev)[: stream.size]
    got = spec_amd.decode_flat(schema, d_stream, to_dev(ends.view(np.int64), dev))
    torch.cuda.synchronize()
    gs = got.status.cpu().numpy()
    if not np.array_equal(gs, want_status):
        i = int(np.nonzero(gs != want_status)[0][0])
        raise AssertionError(f"{label}: status[{i}] gpu={gs[i]} oracle={want_status[i]} "
                             f"record={_rec(stream, ends, i).tobytes().hex()}")
    for f in range(len(schema)):
        g = got.cols[f].cpu().numpy()
        if not np.array_equal(g, want_cols[f]):
            i = int(np.nonzero((g != want_cols[f]).any(axis=1))[0][0])
            raise AssertionError(
                f"{label}: field {f} (tag {schema.fields[f].tag}, {schema.fields[f].kind.name}) "
                f"record {i}: gpu={g[i].tobytes().hex()} oracle={want_cols[f][i].tobytes().hex()} "
                f"record={_rec(stream, ends, i).tobytes().hex()}")
    return got, want_cols, want_status


def check_encode(dev, schema, cols, heaps, n, label=""):
    want_stream, want_ends = oracle_encode(schema, cols, heaps, n)
    d_cols = [to_dev(c, dev) for c in cols]
    d_heaps = {f: to_dev(h if h.size else np.zeros(1, np.uint8), dev) for f, h in heaps.items()}
    out, ends = spec_amd.encode_flat(schema, d_cols, d_heaps, n)
    torch.cuda.synchronize()
    ge = ends.cpu().numpy().view(np.uint64)
    if not np.array_equal(ge, want_ends):
        i = int(np.nonzero(ge != want_ends)[0][0])
        raise AssertionError(f"{label}: ends[{i}] gpu={ge[i]} oracle={want_ends[i]}")
    go = out.cpu().numpy()
    if not np.array_equal(go, want_stream):
        j = int(np.nonzero(go != want_stream)[0][0])
        i = int(np.searchsorted(want_ends, j, side="right"))
        raise AssertionError(f"{label}: byte {j} (record {i}) gpu={go[j]:#x} oracle={want_stream[j]:#x}\n"
                             f"gpu   ={_rec(go, want_ends, i).tobytes().hex()}\n"
                             f"oracle={_rec(want_stream, want_ends, i).tobytes().hex()}")
    return want_stream, want_ends


def _rec(stream, ends, i):
    s = int(ends[i - 1]) if i else 0
    return stream[s:int(ends[i])]


def concat_records(recs):
    """[bytes] -> (stream, ends)"""
    lens = np.array([len(r) for r in recs], dtype=np.uint64)
    ends = np.cumsum(lens, dtype=np.uint64) if len(recs) else np.zeros(0, np.uint64)
    stream = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    return stream, ends


def check_errors(dev, schema, stream: np.ndarray, ends: np.ndarray, label=""):
    """spec_decode_flat_errors vs the oracle: columns, status and the *Err getters' bits."""
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    want_cols, want_status = O.decode_flat_batch(schema.tags, schema.kinds, stream, ends, schema.widths, nthreads=4)
    want_mask = O.decode_flat_errors(schema.tags, schema.kinds, stream, ends)
    d_stream = to_dev(stream if stream.size else np.zeros(1, np.uint8), dev)[: stream.size]
    got, mask = spec_amd.decode_flat_errors(schema, d_stream, to_dev(ends.view(np.int64), dev))
    torch.cuda.synchronize()
    assert np.array_equal(got.status.cpu().numpy(), want_status), f"{label}: status"
    for f in range(len(schema)):
        assert np.array_equal(got.cols[f].cpu().numpy(), want_cols[f]), f"{label}: field {f}"
    gm = mask.cpu().numpy().view(np.uint64)
    assert gm.shape == want_mask.shape, (gm.shape, want_mask.shape)
    if not np.array_equal(gm, want_mask):
        bad = np.argwhere(gm != want_mask)[0]
        i = int(bad[-1])
        raise AssertionError(f"{label}: errmask{tuple(int(b) for b in bad)} gpu={int(gm[tuple(bad)]):x} "
                             f"oracle={int(want_mask[tuple(bad)]):x} "
                             f"record={_rec(stream, ends, i).tobytes().hex()}")
    return gm
