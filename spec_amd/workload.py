"""Synthetic batches for the benchmark and the parity tests.

Flat16 values, seeded numpy PCG64 (seed 0x5EC0DE unless given):
  signed ints   bit length k ~ U[0, width-1], magnitude ~ U[0, 2^k), random sign
  unsigned ints bit length k ~ U[0, width],   value ~ U[0, 2^k)
  floats        finite random bit patterns
  bins          random bytes
  string        ASCII, length ~ U[30, 62];  bytes: random, length ~ U[30, 62]
Mean encoded record ~= 256 B (measured by tests/test_workload.py).

Columns are numpy arrays laid out exactly like the device columns (one uint8 [n, width]
array per field); string/bytes columns are {uint32 off, uint32 len} into per-field heaps.
"""
from __future__ import annotations

import numpy as np

from .schema import FLAT16, Kind, Schema

SEED = 0x5EC0DE


def _signed(rng, n, width):
    k = rng.integers(0, width, size=n)  # bit length in [0, width-1]
    mag = (rng.integers(0, 2**62, size=n, dtype=np.uint64) << np.uint64(2)) | rng.integers(0, 4, size=n, dtype=np.uint64)
    mask = np.where(k >= 64, np.uint64(~np.uint64(0)), (np.uint64(1) << k.astype(np.uint64)) - np.uint64(1))
    mag &= mask
    v = mag.astype(np.int64)
    neg = rng.integers(0, 2, size=n).astype(bool)
    v = np.where(neg, -v, v)
    return v


def _unsigned(rng, n, width):
    k = rng.integers(0, width + 1, size=n)
    v = (rng.integers(0, 2**62, size=n, dtype=np.uint64) << np.uint64(2)) | rng.integers(0, 4, size=n, dtype=np.uint64)
    shift = np.clip(k, 0, 63).astype(np.uint64)
    mask = np.where(k >= 64, np.uint64(~np.uint64(0)), (np.uint64(1) << shift) - np.uint64(1))
    return v & mask


def _finite_bits(rng, n, bits):
    if bits == 32:
        v = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
        exp = (v >> np.uint32(23)) & np.uint32(0xFF)
        v = np.where(exp == 0xFF, v & np.uint32(0xBFFFFFFF), v)  # clear an exponent bit
        return v
    v = (rng.integers(0, 2**62, size=n, dtype=np.uint64) << np.uint64(2)) | rng.integers(0, 4, size=n, dtype=np.uint64)
    exp = (v >> np.uint64(52)) & np.uint64(0x7FF)
    return np.where(exp == 0x7FF, v & np.uint64(0xBFFFFFFFFFFFFFFF), v)


def _heap(rng, n, lo, hi, ascii_only):
    lens = rng.integers(lo, hi + 1, size=n).astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    total = int(lens.sum(dtype=np.uint64))
    if ascii_only:
        heap = rng.integers(32, 127, size=total, dtype=np.uint8)
    else:
        heap = rng.integers(0, 256, size=total, dtype=np.uint8)
    span = np.empty((n, 2), dtype=np.uint32)
    span[:, 0] = offs.astype(np.uint32)
    span[:, 1] = lens
    return span, heap


def as_bytes(a: np.ndarray, n: int) -> np.ndarray:
    a = np.ascontiguousarray(a)
    width = a.dtype.itemsize * (int(np.prod(a.shape[1:])) if a.ndim > 1 else 1)
    return a.view(np.uint8).reshape(n, width)


def gen_columns(schema: Schema, n: int, seed: int = SEED, str_len=(30, 62)):
    """Random values for any flat schema -> (columns [uint8 (n, w)], heaps {field: uint8[]})."""
    rng = np.random.default_rng(seed)
    cols, heaps = [], {}
    for f, fld in enumerate(schema.fields):
        k = fld.kind
        if k == Kind.BOOL:
            a = rng.integers(0, 2, size=n, dtype=np.uint8)
        elif k == Kind.BYTE:
            a = rng.integers(0, 256, size=n, dtype=np.uint8)
        elif k == Kind.INT16:
            a = _signed(rng, n, 16).astype(np.int16)
        elif k == Kind.INT32:
            a = _signed(rng, n, 32).astype(np.int32)
        elif k == Kind.INT64:
            a = _signed(rng, n, 64)
        elif k == Kind.UINT16:
            a = _unsigned(rng, n, 16).astype(np.uint16)
        elif k == Kind.UINT32:
            a = _unsigned(rng, n, 32).astype(np.uint32)
        elif k == Kind.UINT64:
            a = _unsigned(rng, n, 64)
        elif k == Kind.FLOAT32:
            a = _finite_bits(rng, n, 32)
        elif k == Kind.FLOAT64:
            a = _finite_bits(rng, n, 64)
        elif k in (Kind.BIN64, Kind.BIN128, Kind.BIN256):
            a = rng.integers(0, 256, size=(n, fld.width), dtype=np.uint8)
        elif k in (Kind.STRING, Kind.BYTES):
            a, heaps[f] = _heap(rng, n, str_len[0], str_len[1], k == Kind.STRING)
        else:
            raise ValueError(k)
        cols.append(as_bytes(a, n))
    return cols, heaps


def flat16(n: int, seed: int = SEED):
    return gen_columns(FLAT16, n, seed)


def nested(n: int, seed: int = SEED, count=(0, 8), name_len=(8, 24), label_len=(4, 12)):
    """SURVEY.md §8(d) "Nested" (config 4): outer {1 bin128 id, 2 int64 seq, 3 string name,
    4 list<Item>}, Item {1 int32 key, 2 float64 value, 3 string label}.

    Returns a dict of numpy arrays: id [n,16] u8, seq [n] i64, name [n,2] u32 spans into
    name_heap, item_begin [n+1] u32 (CSR), key [m] i32, value [m] f64 (finite bits),
    label [m,2] u32 spans into label_heap."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(count[0], count[1] + 1, size=n).astype(np.uint32)
    item_begin = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(counts, out=item_begin[1:])
    m = int(item_begin[-1])
    name, name_heap = _heap(rng, n, name_len[0], name_len[1], True)
    label, label_heap = _heap(rng, m, label_len[0], label_len[1], True)
    return {
        "id": rng.integers(0, 256, size=(n, 16), dtype=np.uint8),
        "seq": _signed(rng, n, 64),
        "name": name,
        "name_heap": name_heap,
        "item_begin": item_begin,
        "key": _signed(rng, m, 32).astype(np.int32),
        "value": _finite_bits(rng, m, 64).view(np.float64),
        "label": label,
        "label_heap": label_heap,
    }


def _values(rng, kind, m, str_len):
    """m random column elements of a scalar kind -> (uint8 [m, width], heap or None)."""
    k = Kind(kind)
    if k in (Kind.STRING, Kind.BYTES):
        span, heap = _heap(rng, m, str_len[0], str_len[1], k == Kind.STRING)
        return as_bytes(span, m), heap
    sch = Schema([(1, k)])
    cols, _ = gen_columns(sch, m, int(rng.integers(0, 2**63)))
    return cols[0], None


def _any_values(rng, m):
    """Raw encoded values for `any` columns (no varints: the bytes are the same under any
    reverse-varint layout): true/false, byte, float64, or empty (the field is not written)."""
    choice = rng.integers(0, 4, size=m)
    parts, spans, off = [], np.zeros((m, 2), np.uint32), 0
    for i in range(m):
        c = choice[i]
        if c == 0:
            b = bytes([1 if rng.integers(0, 2) else 2])
        elif c == 1:
            b = bytes([int(rng.integers(0, 256)), 3])
        elif c == 2:
            b = rng.integers(0, 256, 8, dtype=np.uint8).tobytes() + bytes([41])
        else:
            b = b""
        spans[i] = (off if b else 0, len(b))
        parts.append(b)
        off += len(b)
    heap = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8).copy()
    return as_bytes(spans, m), heap


def tree_batch(tree, n: int, seed: int = SEED, count=(0, 4), present: float = 0.8, str_len=(0, 20)):
    """Random columns for a spec_amd.Tree (canonical: a field under an absent sub-message or list
    holds zeros, so decode(encode(x)) == x up to span offsets).  Returns (cols {name: uint8
    [entries, width]}, heaps {name: uint8[]}, rows per table)."""
    from .tree import REL_MANY, REL_ONE, ROLE_BEGIN, ROLE_ERRMASK, ROLE_PRESENT, ROLE_STATUS, ROLE_TYPE

    rng = np.random.default_rng(seed)
    T = tree.tables
    rows = [0] * len(T)
    rows[0] = n
    alive = {0: np.ones(n, bool)}
    cols, heaps = {}, {}
    for t in T:
        if t.index:
            f = tree.fields[t.field]
            pres = cols[f"{f.path}?"].reshape(-1).astype(bool)
            if t.rel == REL_ONE:
                rows[t.index] = rows[t.parent]
                alive[t.index] = pres
            else:
                cnt = rng.integers(count[0], count[1] + 1, size=rows[t.parent]).astype(np.uint32) * pres
                begin = np.zeros(rows[t.parent] + 1, np.uint32)
                np.cumsum(cnt, out=begin[1:])
                rows[t.index] = int(begin[-1])
                alive[t.index] = np.ones(rows[t.index], bool)
                cols[f"{f.path}#begin"] = begin.view(np.uint8).reshape(-1, 4)
        R, live = rows[t.index], alive[t.index]
        for c in t.columns:
            if c.role in (ROLE_BEGIN,):
                continue
            if c.role == ROLE_STATUS:
                cols[c.name] = np.zeros((R, 1), np.uint8)
            elif c.role == ROLE_ERRMASK:
                cols[c.name] = np.zeros((R, 8), np.uint8)  # values written by their own kinds: no errors
            elif c.role == ROLE_TYPE:  # Value.Type() of the any value before it: its last byte
                v = tree.fields[c.field].path
                sp, h = cols[v].view(np.uint32).reshape(-1, 2), heaps[v]
                last = np.where(sp[:, 1] > 0, sp[:, 0].astype(np.int64) + sp[:, 1] - 1, 0)
                cols[c.name] = np.where(sp[:, 1] > 0, h[last], 0).astype(np.uint8).reshape(R, 1)
            elif c.role == ROLE_PRESENT:
                cols[c.name] = ((rng.random(R) < present) & live).astype(np.uint8).reshape(R, 1)
            elif c.kind == Kind.ANY:
                a, h = _any_values(rng, R)
                a.view(np.uint32)[~live] = 0
                cols[c.name], heaps[c.name] = a, h
            else:
                a, h = _values(rng, c.kind, R, str_len)
                a[~live] = 0
                cols[c.name] = np.ascontiguousarray(a)
                if h is not None:
                    heaps[c.name] = h if h.size else np.zeros(1, np.uint8)
    return cols, heaps, rows


def bench_wide_schemas():
    """The bench's schemas outside the register-resident fast path (bench.py wide_leg): a
    40-field schema cycling through every kind with its write order permuted, and a 16-field
    schema whose tags > 255 make every table big (internal/format/msg.go:43-61)."""
    from .schema import Kind, Schema

    kinds = [Kind(k) for k in range(1, 16)]
    tags40 = [int(t) for t in np.random.default_rng(3).permutation(np.arange(1, 41))]
    return {"wide40": Schema([(t, kinds[i % 15]) for i, t in enumerate(tags40)]),
            "big16": Schema([(256 + 37 * i, kinds[i % 15]) for i in range(16)])}
