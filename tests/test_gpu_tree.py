"""Schema trees on the GPU (spec_tree_decoder_* / spec_encode_tree) against the oracle's
generated readers/writers (oracle/tree.c): encoded bytes bit-exact, every decoded column
identical (values, PRESENT, BEGIN, STATUS), on pkg1.spec's Message (structs, enum, sub-messages,
recursive Submessage, value lists, struct lists, message lists, any), a tree with lists inside
list items, big tables and big lists, the reference's TestObject, fuzzed and truncated records."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import spec_amd
from spec_amd import workload
from tests.test_tree import _test_object_columns
from tests.trees import many_tables_tree, wide_tree
from tests.tree_helpers import (mismatches, nested_struct_tree, oracle_decode, oracle_encode, roundtrip_mismatches,
                                shapes_tree)

pytestmark = pytest.mark.gpu


def to_dev(d: dict, dev):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items() if v is not None}


def gpu_decode(tree, stream: np.ndarray, ends: np.ndarray, dev):
    s = torch.from_numpy(np.ascontiguousarray(stream) if stream.size else np.zeros(1, np.uint8)).to(dev)[: stream.size]
    e = torch.from_numpy(np.ascontiguousarray(ends).view(np.int64)).to(dev)
    out = spec_amd.decode_tree(tree, s, e)
    torch.cuda.synchronize()
    return out.rows, [c.cpu().numpy() for c in out.cols]


def check_encode_decode(tree, cols, heaps, rows, dev, n):
    want_stream, want_ends = oracle_encode(tree, cols, heaps, n)
    stream, ends = spec_amd.encode_tree(tree, to_dev(cols, dev), to_dev(heaps, dev), n, rows=rows)
    torch.cuda.synchronize()
    assert np.array_equal(ends.cpu().numpy().view(np.uint64), want_ends), "ends"
    assert np.array_equal(stream.cpu().numpy(), want_stream), "encoded bytes"
    want_rows, want = oracle_decode(tree, want_stream, want_ends)
    got_rows, got = gpu_decode(tree, want_stream, want_ends, dev)
    assert got_rows == want_rows == rows
    assert mismatches(tree, got, want) == []
    assert roundtrip_mismatches(tree, cols, heaps, got, want_stream) == []
    return want_stream, want_ends


@pytest.mark.parametrize("n", [1, 7, 1000, 30_000, 131_072])
def test_pkg1_encode_decode(dev, n):
    tree = spec_amd.pkg1_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, 100 + n)
    check_encode_decode(tree, cols, heaps, rows, dev, n)


def _root_windows(ends: np.ndarray, extra: int):
    """The root group's staging per 64-record window, restated from tree_decode.hip group_shape
    and tree_decode_core.hpp tree_rows_pair: the slab (0: no staging), and per window whether its
    span fits the slab (else both waves parse it from HBM) and, for the window holding the stream's
    last partial 16-byte chunk, which wave's 1 KiB DMA chunk it is in (that wave refills it)."""
    n, total = len(ends), int(ends[-1])
    slab = (int(64.0 * total / n * 1.15 + 128 + 64) + 1023) & ~1023
    if slab + extra > 40960:  # WAVE_LDS_MAX
        return 0, []
    starts = np.concatenate([[0], ends[:-1]]).astype(np.int64)
    out = []
    for w in range((n + 63) // 64):
        lo, hi = int(starts[w * 64]), int(ends[min(n, w * 64 + 64) - 1])
        sb, se = max(lo - 64, 0) & ~15, (hi + 31) & ~15
        fits = se - sb + 16 <= slab
        tail, chunks = total & ~15, (se - sb + 1023) >> 10
        tw = ((tail - sb) >> 10) % 2 if fits and total % 16 and sb <= tail < sb + chunks * 1024 else None
        out.append((fits, tw))
    return slab, out


@pytest.mark.parametrize("case", ["tail_wave0", "tail_wave1", "last_over_slab"])
def test_pkg1_root_pair_over_slab_and_stream_end(dev, case):
    """The root group on wave pairs (tree_rows_pair) at the two edges its staging has: a 64-record
    window whose span exceeds the slab (both waves parse it from HBM, range-checked) among staged
    windows, and the window holding the stream's last partial 16-byte chunk, which comes back
    zeroed from the LDS-DMA and is refilled bytewise by the wave whose round-robin 1 KiB chunk
    holds it (wave 0 or wave 1), or, in the third case, that last window over the slab itself.
    The records are a pkg1 batch rearranged (records are independent): window 1 (or the last
    window) is 64 copies of the batch's largest record; the record count is chosen so the
    windows land as the case needs, and the test asserts they do.  Against the oracle's decode of
    the same stream (round 5's first pair-kernel run, gpurun_out/pair1, failed pkg1 at 131,072
    records with 41 columns wrong; DESIGN.md §3.7 "pair1")."""
    from spec_amd.tree import REL_ONE

    tree = spec_amd.pkg1_tree()
    cols, heaps, rows = workload.tree_batch(tree, 1500, 77)
    s, e = oracle_encode(tree, cols, heaps, 1500)
    e = e.astype(np.int64)
    st = np.concatenate([[0], e[:-1]])
    sz = e - st
    big = int(np.argmax(sz))
    gn = 1 + sum(1 for t in tree.tables if t.index and t.rel == REL_ONE and tree.tables[t.parent].rel != 2)
    extra = 512 * (gn - 1) + 16
    pick = None
    for m in range(600, 1500):
        order = list(range(64)) + [big] * 64 + list(range(128, m))
        if case == "last_over_slab":
            order = list(range(m - 64)) + [big] * 64
        slab, w = _root_windows(np.cumsum(sz[order]), extra)
        if not slab:
            continue
        if case == "last_over_slab":
            ok = not w[-1][0] and all(f for f, _ in w[:-1]) and int(np.sum(sz[order])) % 16
        else:
            ok = not w[1][0] and all(f for f, _ in w[:1] + w[2:]) and w[-1][1] == int(case[-1])
        if ok:
            pick = order
            break
    assert pick is not None, "no record count puts the windows where the case needs them"
    stream = np.concatenate([s[st[i]: e[i]] for i in pick])
    ends = np.cumsum(sz[pick]).astype(np.uint64)
    want_rows, want = oracle_decode(tree, stream, ends)
    got_rows, got = gpu_decode(tree, stream, ends, dev)
    assert got_rows == want_rows
    assert mismatches(tree, got, want) == []


@pytest.mark.parametrize("n,str_len", [(200, (0, 3000)), (3, (80_000, 100_000)), (130, (0, 600))])
def test_pkg1_tiles_over_the_image(dev, n, str_len):
    """The record-tile writer (jit.cpp gen_tile) on tiles whose output range exceeds its LDS image
    (36 KiB at 4 waves per workgroup): the bytes past the image's window go straight to HBM (tree_core.hpp LSink), whether
    64 records add up past it (25 KB records) or one record alone does (a 100 KB string), and a
    batch whose last tile is partial (130 records)."""
    tree = spec_amd.pkg1_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, 500 + n, str_len=str_len)
    stream, ends = check_encode_decode(tree, cols, heaps, rows, dev, n)
    starts = np.concatenate([[0], ends[:-1]]).astype(np.int64)
    tiles = [int(ends[min(n, t + 64) - 1]) - int(starts[t]) for t in range(0, n, 64)]
    assert max(tiles) > 72 * 1024 or str_len[1] < 1000  # past the image at any TREE_TILE_W


@pytest.mark.parametrize("depth", [1, 3])
def test_pkg1_depths(dev, depth):
    tree = spec_amd.pkg1_tree(depth)
    cols, heaps, rows = workload.tree_batch(tree, 500, depth, present=0.9)
    check_encode_decode(tree, cols, heaps, rows, dev, 500)


def test_shapes_big_lists_big_tables(dev):
    tree = shapes_tree()
    cols, heaps, rows = workload.tree_batch(tree, 60, 9, count=(0, 300), str_len=(0, 70))
    assert max(rows) > 255
    check_encode_decode(tree, cols, heaps, rows, dev, 60)


def test_shapes_many_small(dev):
    tree = shapes_tree()
    cols, heaps, rows = workload.tree_batch(tree, 5000, 10, count=(0, 3))
    check_encode_decode(tree, cols, heaps, rows, dev, 5000)


def test_test_object(dev):
    tree = spec_amd.pkg1_tree()
    cols, heaps = _test_object_columns(tree)
    rows = spec_amd.tree_rows(tree, 1, cols)
    check_encode_decode(tree, cols, heaps, rows, dev, 1)


def test_empty_batch(dev):
    tree = spec_amd.pkg1_tree()
    rows, got = gpu_decode(tree, np.zeros(0, np.uint8), np.zeros(0, np.uint64), dev)
    assert rows == [0] * len(tree.tables)


@pytest.mark.parametrize("seed", range(4))
def test_fuzzed_records(dev, seed):
    """Mutated, truncated and garbage records: every status class, panics, nil elements —
    identical to the oracle column for column."""
    tree = spec_amd.pkg1_tree() if seed % 2 == 0 else shapes_tree()
    n = 2000
    cols, heaps, rows = workload.tree_batch(tree, n, 200 + seed, count=(0, 5))
    stream, ends = oracle_encode(tree, cols, heaps, n)
    rng = np.random.default_rng(seed)
    s = stream.copy()
    k = max(1, s.size // 200)
    idx = rng.integers(0, s.size, k)
    s[idx] = rng.integers(0, 256, k, dtype=np.uint8)
    e = ends.copy()
    cut = rng.integers(0, n, n // 20)
    starts = np.concatenate([[0], e[:-1]])
    e[cut] = np.maximum(starts[cut], e[cut] - rng.integers(0, 5, cut.size).astype(np.uint64))  # truncated records
    want_rows, want = oracle_decode(tree, s, e)
    got_rows, got = gpu_decode(tree, s, e, dev)
    assert got_rows == want_rows
    assert mismatches(tree, got, want) == []


def _fuzz(stream, ends, seed, n):
    rng = np.random.default_rng(seed)
    s = stream.copy()
    k = max(1, s.size // 200)
    idx = rng.integers(0, s.size, k)
    s[idx] = rng.integers(0, 256, k, dtype=np.uint8)
    e = ends.copy()
    cut = rng.integers(0, n, n // 20)
    starts = np.concatenate([[0], e[:-1]])
    e[cut] = np.maximum(starts[cut], e[cut] - rng.integers(0, 5, cut.size).astype(np.uint64))
    return s, e


@pytest.mark.parametrize("n", [1, 300, 20_000])
def test_nested_structs_encode_decode(dev, n):
    """Structs inside structs (internal/lang/model/struct_field.go:57-70; generated Decode /
    EncodeXxxTo recurse, generator/struct.go:75-142): in a message, in a list, in a sub-message,
    three levels deep; encode bit-exact, decode identical to the oracle."""
    tree = nested_struct_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, 300 + n)
    check_encode_decode(tree, cols, heaps, rows, dev, n)


@pytest.mark.parametrize("seed", range(3))
def test_nested_structs_fuzzed(dev, seed):
    """Mutated and truncated nested-struct records: inner struct errors stop the outer decode,
    panics at any depth — identical to the oracle column for column."""
    tree = nested_struct_tree()
    n = 3000
    cols, heaps, rows = workload.tree_batch(tree, n, 400 + seed, count=(0, 4))
    stream, ends = oracle_encode(tree, cols, heaps, n)
    s, e = _fuzz(stream, ends, 40 + seed, n)
    want_rows, want = oracle_decode(tree, s, e)
    got_rows, got = gpu_decode(tree, s, e, dev)
    assert got_rows == want_rows
    assert mismatches(tree, got, want) == []


@pytest.mark.parametrize("n", [1, 300, 5000])
def test_wide_encode_decode(dev, n):
    """More than 64 direct fields (internal/format/msg.go:13-61 takes any number of u16 tags):
    a 130-field record with a big table, a 70-member struct, an 80-field sub-message and list
    item — encode bit-exact (generated writers), decode identical to the oracle (the run-time
    group kernel: multi-word ERRMASK)."""
    tree = wide_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, 500 + n, count=(0, 3))
    check_encode_decode(tree, cols, heaps, rows, dev, n)


@pytest.mark.parametrize("seed", range(2))
def test_wide_fuzzed(dev, seed):
    """Mutated and truncated 130-field records: the *Err bits of fields past 64 (ERRMASK words
    1 and 2) identical to the oracle's."""
    tree = wide_tree()
    n = 1500
    cols, heaps, rows = workload.tree_batch(tree, n, 600 + seed, count=(0, 3))
    stream, ends = oracle_encode(tree, cols, heaps, n)
    s, e = _fuzz(stream, ends, 60 + seed, n)
    want_rows, want = oracle_decode(tree, s, e)
    got_rows, got = gpu_decode(tree, s, e, dev)
    assert got_rows == want_rows
    assert mismatches(tree, got, want) == []
    em = {c.name: w for c, w in zip(tree.columns, want)}["#errmask"].view(np.uint64)
    assert em.shape[1] == 3 and em[:, 1:].any()  # errors reported past the first 64 fields


@pytest.mark.parametrize("n", [1, 2000])
def test_many_tables_encode_decode(dev, n):
    """114 tables (100 sub-message range slots in the records' decode group: fewer waves per
    workgroup) and a struct chain 14 deep: encode bit-exact, decode identical to the oracle."""
    tree = many_tables_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, 700 + n, count=(0, 3))
    check_encode_decode(tree, cols, heaps, rows, dev, n)


def test_many_tables_fuzzed(dev):
    tree = many_tables_tree()
    n = 800
    cols, heaps, rows = workload.tree_batch(tree, n, 707, count=(0, 3))
    stream, ends = oracle_encode(tree, cols, heaps, n)
    s, e = _fuzz(stream, ends, 71, n)
    want_rows, want = oracle_decode(tree, s, e)
    got_rows, got = gpu_decode(tree, s, e, dev)
    assert got_rows == want_rows
    assert mismatches(tree, got, want) == []


def test_encoder_error_span_outside_heap(dev):
    tree = spec_amd.pkg1_tree()
    cols, heaps, rows = workload.tree_batch(tree, 10, 3)
    cols = dict(cols)
    bad = cols["string"].copy()
    bad.view(np.uint32)[3, 0] = 1 << 30
    cols["string"] = bad
    enc = spec_amd.TreeEncoder(tree, rows, dev)
    total = enc.encode(to_dev(cols, dev), to_dev(heaps, dev), None, None)
    assert int(total.item()) == -1


@pytest.mark.parametrize("name", ["pkg1.Message", "pmpx.Message", "prpc.Message", "pmpx.ChannelOpen"])
def test_reference_spec_trees(dev, name):
    """Trees the .spec front end derives from the reference's own schemas (fixture made by
    tests/golden/make_spec_trees.py from pkg1.spec, proto/pmpx/mpx.spec, proto/prpc/rpc.spec)."""
    import json
    import os

    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "spec_trees.json")))
    tree = spec_amd.Tree.from_fields(d[name])
    cols, heaps, rows = workload.tree_batch(tree, 3000, 77, count=(0, 3))
    check_encode_decode(tree, cols, heaps, rows, dev, 3000)


@pytest.mark.parametrize("name", ["pmpx.Message", "pkg1.Message"])
def test_reference_spec_trees_at_scale(dev, name):
    """100k-record batches of the reference's own schemas (pmpx.Message from proto/pmpx/mpx.spec,
    pkg1.Message from internal/tests/pkg1/pkg1.spec) through the .spec-derived trees."""
    import json
    import os

    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "spec_trees.json")))
    tree = spec_amd.Tree.from_fields(d[name])
    n = 100_000
    cols, heaps, rows = workload.tree_batch(tree, n, 91, count=(0, 4))
    check_encode_decode(tree, cols, heaps, rows, dev, n)


@pytest.mark.parametrize("shift", [1, 4, 9])
def test_errmask_cross_kind(dev, shift):
    """Per-row *Err masks (ERRMASK columns) of every message table: records written by pkg1's
    writer and read through a tree whose scalar fields have other kinds (range / type errors at
    every level: records, sub-messages, list items), plus ListErr / MessageErr / struct /
    OpenValueErr bits from fuzzed bytes — identical to the oracle's *Err getters."""
    tree = spec_amd.pkg1_tree()
    n = 3000
    cols, heaps, rows = workload.tree_batch(tree, n, 500 + shift, count=(0, 3))
    stream, ends = oracle_encode(tree, cols, heaps, n)
    fields = []
    for p, tag, k, e, par in tree.to_fields():
        if 1 <= k <= 15:
            k = (k - 1 + shift) % 15 + 1
        fields.append((p, tag, k, e, par))
    reader = spec_amd.Tree.from_fields(fields)
    for s, e in ((stream, ends), _fuzz(stream, ends, shift, n)):
        want_rows, want = oracle_decode(reader, s, e)
        got_rows, got = gpu_decode(reader, s, e, dev)
        assert got_rows == want_rows
        assert mismatches(reader, got, want) == []
    masks = [g for c, g in zip(reader.columns, got) if c.name.endswith("#errmask")]
    assert any(np.any(m) for m in masks)


def _spec_tree(name):
    import json
    import os

    d = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "spec_trees.json")))
    return spec_amd.Tree.from_fields(d[name])


def test_any_message_field_as_sub_table(dev):
    """pkg1.spec `message1 message 52` (internal/tests/pkg1/pkg1.spec:30): the generated getter is
    m.msg.Field(52).Message() (generator/message.go:145-148) — an `any` span, then OpenMessage
    over it (Value.Message, internal/types/value.go:318-321).  The span column of the record
    decode feeds a second tree decode (spec_tree_decoder_index_spans) under the caller's schema
    for it; identical to the oracle's OpenValue(...).Message() + getters, and the values written
    come back."""
    from oracle import oracle as O
    from spec_amd import Kind
    from spec_amd.tree import ListOf, Message

    tree = _spec_tree("pkg1.Message")
    assert tree.column("message1").kind == Kind.ANY
    sub = spec_amd.Tree(Message("message1", [("f1", 1, Kind.INT32), ("f2", 2, Kind.INT32),
                                             ("f3", 3, Kind.INT32), ("l", 4, ListOf(Kind.STRING))]))
    n = 4000
    scols, sheaps, srows = workload.tree_batch(sub, n, 31, count=(0, 3))
    sub_stream, sub_ends = oracle_encode(sub, scols, sheaps, n)
    cols, heaps, rows = workload.tree_batch(tree, n, 32, count=(0, 2))
    starts = np.concatenate([[0], sub_ends[:-1]]).astype(np.uint32)
    sp = np.stack([starts, (sub_ends - starts).astype(np.uint32)], 1)
    empty = np.random.default_rng(5).random(n) < 0.1  # the field not written
    sp[empty] = 0
    cols["message1"] = sp.astype(np.uint32).view(np.uint8)
    heaps["message1"] = sub_stream
    cols["message1#type"] = np.where(sp[:, 1] > 0, 0x50, 0).astype(np.uint8).reshape(n, 1)
    stream, ends = check_encode_decode(tree, cols, heaps, rows, dev, n)
    # the record decode's message1 spans (oracle == GPU, checked above)
    _, want = oracle_decode(tree, stream, ends)
    spans = want[tree.column("message1").index]
    want_rows, want_sub = O.decode_tree_spans(tree_fields_of(sub), stream, spans)
    d = spec_amd.TreeDecoder(sub)
    got_rows = d.index_spans(torch.from_numpy(stream).to(dev), torch.from_numpy(np.ascontiguousarray(spans)).to(dev))
    got = [c.cpu().numpy() for c in d.decode().cols]
    torch.cuda.synchronize()
    assert got_rows == want_rows
    assert mismatches(sub, got, want_sub) == []
    g = {c.name: v for c, v in zip(sub.columns, got)}
    assert np.array_equal(g["f1"][~empty], scols["f1"][~empty]) and not g["f1"][empty].any()
    assert not g["#status"].any()


def tree_fields_of(tree):
    from tests.tree_helpers import oracle_fields

    return oracle_fields(tree)


@pytest.mark.parametrize("seed", range(2))
def test_typed_values_of_any(dev, seed):
    """Value.<Kind>() / <Kind>Err() (internal/types/value.go:120-310) over pkg1's `any` spans for
    every kind (type errors where the value has another type), spans past the stream, fuzzed
    bytes — spec_decode_values == the oracle."""
    from oracle import oracle as O
    from spec_amd import Kind

    tree = spec_amd.pkg1_tree()
    n = 3000
    cols, heaps, rows = workload.tree_batch(tree, n, 600 + seed)
    stream, ends = oracle_encode(tree, cols, heaps, n)
    if seed:
        stream, _ = _fuzz(stream, ends, seed, n)
    _, want = oracle_decode(tree, stream, ends)
    spans = np.ascontiguousarray(want[tree.column("any").index]).view(np.uint32).reshape(-1, 2).copy()
    spans[::97] = (len(stream) - 3, 9)  # past the stream: a Go panic
    d_stream = torch.from_numpy(stream).to(dev)
    d_spans = torch.from_numpy(spans).to(dev)
    for k in range(1, 16):
        wv, we = O.decode_values(k, stream, spans)
        gv, ge = spec_amd.decode_values(Kind(k), d_stream, d_spans)
        torch.cuda.synchronize()
        assert np.array_equal(ge.cpu().numpy(), we), Kind(k)
        assert np.array_equal(gv.cpu().numpy(), wv), Kind(k)


def test_run_async_and_capacity(dev):
    """spec_tree_decoder_run: a new batch decoded in one pass with no host synchronisation, row
    counts on the device == index(); a batch whose lists outgrow the capacity reports -1 for
    those tables (and decodes the rest), then fits after reserve()."""
    tree = spec_amd.pkg1_tree()
    small_cols, small_heaps, _ = workload.tree_batch(tree, 500, 71, count=(0, 2))
    s1, e1 = oracle_encode(tree, small_cols, small_heaps, 500)
    cols, heaps, rows = workload.tree_batch(tree, 500, 72, count=(3, 6))
    s2, e2 = oracle_encode(tree, cols, heaps, 500)
    want_rows, want = oracle_decode(tree, s2, e2)
    d = spec_amd.TreeDecoder(tree)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d.index(to(s1), to(e1.view(np.int64)))               # sizes the lists for the small batch
    out = [torch.zeros((max(tree.column_rows(c, want_rows), 1), c.width), dtype=torch.uint8, device=dev)
           for c in tree.columns]
    got_rows = d.run(to(s2), to(e2.view(np.int64)), out).cpu().numpy()
    lists = [t.index for t in tree.tables if t.rel == 2]
    assert all(got_rows[t] == -1 for t in lists if want_rows[t] > d.rows[t] * 9 // 8 + 64)
    d.reserve(want_rows)
    got_rows = d.run(to(s2), to(e2.view(np.int64)), out).cpu().numpy()
    assert list(got_rows) == want_rows
    got = [c[: tree.column_rows(tc, want_rows)].cpu().numpy() for c, tc in zip(out, tree.columns)]
    assert mismatches(tree, got, want) == []


def test_run_columns_sized_by_indexed_batch(dev):
    """columns allocated from an indexed batch's rows, then a batch with more
    list elements run into them — within the decoder's internal capacity (index grows it by 1/8
    + 64), beyond the columns.  Nothing may be written past a column: each column sits between
    guard bytes that must stay intact; lists that do not fit (and tables under them) report -1,
    every other table decodes exactly."""
    tree = spec_amd.pkg1_tree()
    cols_a, heaps_a, _ = workload.tree_batch(tree, 400, 81, count=(3, 4))
    s1, e1 = oracle_encode(tree, cols_a, heaps_a, 400)
    cols_b, heaps_b, _ = workload.tree_batch(tree, 400, 82, count=(4, 4))
    s2, e2 = oracle_encode(tree, cols_b, heaps_b, 400)
    want_rows, want = oracle_decode(tree, s2, e2)
    d = spec_amd.TreeDecoder(tree)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    rows_a = d.index(to(s1), to(e1.view(np.int64)))
    caps = d.capacity()
    lists = [t.index for t in tree.tables if t.rel == 2]
    assert any(rows_a[t] < want_rows[t] <= caps[t] for t in lists)  # the case the advice describes
    guard = 4096
    bufs, out = [], []
    for c in tree.columns:
        nbytes = max(tree.column_rows(c, rows_a), 1) * c.width
        b = torch.full((nbytes + 2 * guard,), 0xA5, dtype=torch.uint8, device=dev)
        bufs.append((b, nbytes))
        out.append(b[guard: guard + nbytes].view(-1, c.width))
    got_rows = d.run(to(s2), to(e2.view(np.int64)), out).cpu().numpy()
    torch.cuda.synchronize()
    for (b, nbytes), c in zip(bufs, tree.columns):
        h = b.cpu().numpy()
        assert (h[:guard] == 0xA5).all() and (h[guard + nbytes:] == 0xA5).all(), c.name

    over = {t for t in lists if want_rows[t] > rows_a[t]}

    def under(t):  # t is, or hangs under, a list that did not fit
        while t > 0:
            if t in over:
                return True
            t = tree.tables[t].parent
        return False

    assert over
    for t in range(len(tree.tables)):
        assert got_rows[t] == (-1 if under(t) else want_rows[t]), t
    for i, c in enumerate(tree.columns):
        if not under(c.table):
            g = out[i][: tree.column_rows(c, want_rows)].cpu().numpy()
            assert np.array_equal(g, want[i]), c.name


def test_rows_out_first_run_without_index(dev):
    """run() on a fresh decoder (no index, list capacities 0) reports -1 for
    every list table (none fits), never uninitialised counts."""
    tree = spec_amd.pkg1_tree()
    cols, heaps, _ = workload.tree_batch(tree, 300, 83)
    s, e = oracle_encode(tree, cols, heaps, 300)
    want_rows, _ = oracle_decode(tree, s, e)
    d = spec_amd.TreeDecoder(tree)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    out = [torch.zeros((max(tree.column_rows(c, want_rows), 1), c.width), dtype=torch.uint8, device=dev)
           for c in tree.columns]
    got = d.run(to(s), to(e.view(np.int64)), out).cpu().numpy()
    for t, tb in enumerate(tree.tables):
        if tb.rel == 2 or (t and got[tb.parent] == -1):
            assert got[t] == -1 or want_rows[t] == 0, (t, got[t], want_rows[t])
        elif t and tree.tables[t].parent == 0:
            assert got[t] == 300


def test_list_scan_many_tiles(dev):
    """Owner rows over 1,024 scan tiles (1,100,000 records): the list scans take the top-level
    offset launch (list_top_kernel, m.top) instead of per-block sums of the earlier tiles; both
    paths give the oracle's BEGIN columns and element rows."""
    from spec_amd.schema import Kind
    from spec_amd.tree import ListOf, Message, Tree

    tree = Tree(Message("message1", [("f1", 1, Kind.INT32), ("f2", 2, Kind.INT32), ("f3", 3, Kind.INT32),
                                     ("l", 4, ListOf(Kind.STRING))]))  # tree_catalog's last tree (precompiled)
    n = 1_100_000
    cols, heaps, rows = workload.tree_batch(tree, n, 21, count=(0, 3), str_len=(0, 6))
    check_encode_decode(tree, cols, heaps, rows, dev, n)


def pad_list_rows(tree, cols, rows, x, front, back, per=2):
    """The batch (cols, rows) with list table x given `front` rows before and `back` rows after
    the range its owners' BEGIN cover (begin[0] > 0, rows past begin[owner rows]).  Every table
    under x gets matching junk rows: a REL_ONE child one per junk owner row, a list `per`
    elements per junk owner row (covered by that list's own BEGIN range, owned by a junk row).
    Junk rows copy row 0's values (valid spans: the size pass checks every row).  The batch
    encodes to the same bytes as the original: nothing under an uncovered row is written."""
    from spec_amd.tree import REL_ONE, ROLE_BEGIN, INPUT_ROLES

    cols, rows = dict(cols), list(rows)
    pad = {x: (front, back)}
    bname = f"{tree.fields[tree.tables[x].field].path}#begin"
    cols[bname] = (cols[bname].reshape(-1).view(np.uint32) + np.uint32(front)).view(np.uint8).reshape(-1, 4)
    for t in tree.tables[x + 1:]:  # pre-order: owners first
        if t.parent not in pad:
            continue
        F, K = pad[t.parent]
        if t.rel == REL_ONE:
            pad[t.index] = (F, K)
            continue
        bn = f"{tree.fields[t.field].path}#begin"
        b = cols[bn].reshape(-1).view(np.uint32).astype(np.int64)
        Fc = F * per
        nb = np.concatenate([np.arange(0, Fc, per), b + Fc, b[-1] + Fc + per * np.arange(1, K + 1)])
        cols[bn] = nb.astype(np.uint32).view(np.uint8).reshape(-1, 4)
        pad[t.index] = (Fc, K * per)
    for t, (F, K) in pad.items():
        for c in tree.tables[t].columns:
            if c.role == ROLE_BEGIN or c.role not in INPUT_ROLES or c.name not in cols:
                continue
            a = cols[c.name].reshape(rows[t], c.width)
            tmpl = a[:1] if rows[t] else np.zeros((1, c.width), np.uint8)
            cols[c.name] = np.ascontiguousarray(np.concatenate([np.repeat(tmpl, F, 0), a, np.repeat(tmpl, K, 0)]))
        rows[t] += F + K
    return cols, rows


@pytest.mark.parametrize("which", ["pkg1_3", "shapes"])
def test_encode_list_rows_outside_owner_ranges(dev, which):
    """list rows outside their owners' BEGIN ranges (begin[0] > 0, trailing
    rows) are skipped by the level-fused writers, and so is everything under them — their
    sub-message rows and nested list rows get no position.  The workspace is zero-filled before
    the call (a stale position 0 would write over the first record), and bytes past the output
    capacity stay intact: the output == the oracle Writer's bytes of the unpadded batch."""
    from spec_amd.tree import REL_MANY, SHAPE_MESSAGE

    tree = spec_amd.pkg1_tree(3) if which == "pkg1_3" else shapes_tree()
    n = 400
    cols, heaps, rows = workload.tree_batch(tree, n, 1234, count=(1, 3), present=0.9)
    want_stream, want_ends = oracle_encode(tree, cols, heaps, n)
    lists = [t.index for t in tree.tables if t.rel == REL_MANY and t.shape == SHAPE_MESSAGE and t.parent == 0]
    assert lists
    for x in lists:
        pcols, prows = pad_list_rows(tree, cols, rows, x, 3, 5)
        enc = spec_amd.TreeEncoder(tree, prows, dev)
        enc.workspace.zero_()
        total = int(enc.encode(to_dev(pcols, dev), to_dev(heaps, dev), None, None).item())
        assert total == want_stream.size, x
        guard = 4096
        buf = torch.full((total + guard,), 0xA5, dtype=torch.uint8, device=dev)
        ends = torch.zeros(n, dtype=torch.int64, device=dev)
        enc.workspace.zero_()
        enc.encode(to_dev(pcols, dev), to_dev(heaps, dev), buf[:total], ends)
        torch.cuda.synchronize()
        b = buf.cpu().numpy()
        assert (b[total:] == 0xA5).all(), x
        assert np.array_equal(b[:total], want_stream), x
        assert np.array_equal(ends.cpu().numpy().view(np.uint64), want_ends), x
