"""GPU parity for list<message> decode (BASELINE config 4) against the CPU oracle: outer
columns + status, the item_begin index and item columns + item status, bit for bit."""
from __future__ import annotations

import os

import numpy as np
import pytest

import spec_amd
from oracle import oracle as O
from spec_amd import NESTED, Kind, workload
from tests.gpu_helpers import concat_records, to_dev

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(params=["jit", "generic"])
def kernel(request):
    """Schema-specialised one-pass kernel (hiprtc) and the precompiled generic kernels."""
    spec_amd.set_jit(request.param == "jit")
    yield request.param
    spec_amd.set_jit(True)


MODE_IDS = {"twopass": 1, "twopass-ranges": 2, "twopass-halves": 3, "twopass-tail": 4, "twopass-xcd": 5}


def check_nested(dev, stream, ends, label="",
                 modes=("twopass", "twopass-ranges", "twopass-halves", "twopass-tail", "twopass-xcd", "onepass", "onepass-small-cap")):
    """Every decode mode against the oracle: index + decode (items found by the owner search,
    items from precomputed LDS ranges, half-group slabs, the count pass from tail windows vs
    the staged-span count, XCD-aware decode order: spec_set_nested_mode 1 / 2 / 3 / 4 / 5), one pass with room for
    every item, one pass that first runs out of item room (and decodes again with the total)."""
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    want = O.decode_nested_batch(stream, ends)
    d_stream = to_dev(stream if stream.size else np.zeros(1, np.uint8), dev)[: stream.size]
    d_ends = to_dev(ends.view(np.int64), dev)
    got = None
    L = spec_amd.lib()
    for mode in modes:
        cap = 1 if mode == "onepass-small-cap" else None
        L.spec_set_nested_mode(MODE_IDS.get(mode, 5))
        try:
            got = _check_nested_mode(dev, d_stream, d_ends, want, len(ends), f"{label} [{mode}]",
                                     onepass=not mode.startswith("twopass"), item_cap=cap)
        finally:
            L.spec_set_nested_mode(5)
    return got, want


def _check_nested_mode(dev, d_stream, d_ends, want, n, label, onepass, item_cap):
    import torch

    got = spec_amd.decode_nested(NESTED, d_stream, d_ends, onepass=onepass, item_cap=item_cap)
    torch.cuda.synchronize()
    assert np.array_equal(got.status.cpu().numpy(), want["status"]), label + ": status"
    assert np.array_equal(got.item_begin.cpu().numpy().view(np.uint32), want["item_begin"]), label + ": item_begin"
    m = int(want["item_begin"][-1]) if n else 0
    assert got.total_items == m, label
    assert np.array_equal(got.outer[0].cpu().numpy(), want["id"]), label + ": id"
    assert np.array_equal(got.outer[1].cpu().numpy().view(np.int64).ravel(), want["seq"]), label + ": seq"
    assert np.array_equal(got.outer[2].cpu().numpy().view(np.uint32), want["name"]), label + ": name"
    if m:
        assert np.array_equal(got.item_status.cpu().numpy()[:m], want["item_status"]), label + ": item_status"
        assert np.array_equal(got.items[0][:m].cpu().numpy().view(np.int32).ravel(), want["key"]), label + ": key"
        assert np.array_equal(got.items[1][:m].cpu().numpy().view(np.uint64).ravel(),
                              want["value"].view(np.uint64)), label + ": value"
        assert np.array_equal(got.items[2][:m].cpu().numpy().view(np.uint32), want["label"]), label + ": label"
    return got


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 5000])
def test_nested_parity(dev, kernel, n):
    w = workload.nested(n, seed=n)
    stream, ends = O.encode_nested_batch(w)
    check_nested(dev, stream, ends, f"nested n={n}")


@pytest.mark.parametrize("name_len", [(330, 368), (300, 330), (360, 420)])
def test_nested_large_records_generic(dev, name_len):
    """Mean records of ~510-600 B on the precompiled generic kernels: the slab a 4-wave block
    would need crosses the 160 KiB LDS of a workgroup around 545 B, where the nested slab falls
    back to 0 (parse from HBM) instead of failing the launch."""
    spec_amd.set_jit(False)
    try:
        w = workload.nested(3000, seed=len(name_len) + name_len[0], name_len=name_len)
        stream, ends = O.encode_nested_batch(w)
        check_nested(dev, stream, ends, f"large records {name_len}")
    finally:
        spec_amd.set_jit(True)


@pytest.mark.parametrize("big_at,shape", [(0, "huge"), (5, "double"), (15, "huge"), (15, "double")])
def test_nested_pair_group_over_slab(dev, big_at, shape):
    """The two-pass decode runs a wave pair per group (nested_decode_pair): one group of 64 records
    with long lists in a batch of short ones is larger than the slab sized from the batch's mean,
    so that group goes to wave 0 alone in two halves (or from HBM) while its neighbours run on
    pairs; item offsets on both sides of it must still line up.  "double": ~2x the mean record
    (each half of the group fits the slab); "huge": ~14x (the halves parse from HBM)."""
    small = workload.nested(1024, seed=40 + big_at)
    count, label_len = ((40, 60), (20, 40)) if shape == "huge" else ((6, 9), (6, 12))
    big = workload.nested(64, seed=41 + big_at, count=count, label_len=label_len)
    s1, e1 = O.encode_nested_batch(small)
    s2, e2 = O.encode_nested_batch(big)
    e1 = e1.astype(np.uint64)
    e2 = e2.astype(np.uint64)
    k = 64 * big_at  # the big group's first record
    cut = int(e1[k - 1]) if k else 0
    stream = np.concatenate([s1[:cut], s2, s1[cut:]])
    ends = np.concatenate([e1[:k], e2 + np.uint64(cut), e1[k:] + np.uint64(s2.size)])
    check_nested(dev, stream, ends, f"big group {big_at} {shape}", modes=("twopass", "twopass-xcd", "onepass"))


def test_nested_golden(dev):
    g = np.load(os.path.join(GOLDEN, "nested_small.npz"), allow_pickle=False)
    got, _ = check_nested(dev, g["stream"], g["ends"], "golden")
    assert np.array_equal(got.item_begin.cpu().numpy().view(np.uint32), g["out_item_begin"])


def test_nested_full_size(dev):
    """BASELINE config 4 at full size: 1M records."""
    n = 1 << 20
    w = workload.nested(n)
    stream, ends = O.encode_nested_batch(w)
    check_nested(dev, stream, ends, "nested 1M")


def _record(items, name="nm", list_tag=4, extra=None):
    wr = O.Writer()
    wr.message()
    wr.field(1, "bin128", bytes(range(16)))
    wr.field(2, "int64", -7)
    wr.field(3, "string", name)
    if items is not None:
        wr.field_list(list_tag)
        for k, v, lab in items:
            wr.elem_message()
            wr.field(1, "int32", k)
            wr.field(2, "float64", v)
            wr.field(3, "string", lab)
            assert wr.end()[1] is None
        assert wr.end()[1] is None
    if extra:
        for tag, kind, v in extra:
            wr.field(tag, kind, v)
    b, err = wr.end()
    assert err is None, err
    return b


def test_nested_edge_cases(dev, kernel):
    """No list field, empty list, a big list (> 255 items), the list under another tag, items
    with missing/extra fields, garbage records and truncated records."""
    recs = [
        _record(None),
        _record([]),
        _record([(i, i * 0.5, "x" * (i % 7)) for i in range(300)]),
        _record([(1, 1.0, "a")], list_tag=9),
        _record([(2, 2.0, "bb"), (3, -3.0, "")], extra=[(5, "int32", 1)]),
        b"",
        bytes([1, 2, 3, 80]),
    ]
    good = _record([(4, 4.0, "cccc")] * 3)
    recs.append(good[: len(good) // 2])
    recs.append(good)
    # item messages written by hand: item with only field 2, item that is an int64 not a message
    wr = O.Writer()
    wr.message()
    wr.field_list(4)
    wr.elem_message()
    wr.field(2, "float64", 9.5)
    wr.end()
    wr.elem_int64(12345)
    wr.end()
    b, err = wr.end()
    assert err is None
    recs.append(b)
    stream, ends = concat_records(recs * 20)
    check_nested(dev, stream, ends, "edge")


def test_nested_malformed_list_tables(dev, kernel):
    """List tables whose element ends decrease (Go panics on the slice => SPEC_STATUS_PANIC
    for that item) or exceed the list's data size (nil items)."""
    item = _record([(1, 1.0, "a")])
    # build list bytes by hand: two items, then a table with swapped ends
    it1, _, _ = O.encode("int64", 5)
    it2, _, _ = O.encode("int64", 6)
    data = it1 + it2
    for offs in ([len(data), len(it1)], [len(it1), len(data) + 100], [len(it1), len(data)]):
        lst_trailer, _, err = O.encode_list_table(len(data), offs)
        assert err is None
        lst = data + lst_trailer
        fields = [(4, len(lst))]
        msg_trailer, _, _ = O.encode_message_table(len(lst), fields)
        rec = lst + msg_trailer
        stream, ends = concat_records([item, rec, item] * 30)
        check_nested(dev, stream, ends, f"malformed {offs}")


@pytest.mark.parametrize("seed", range(4))
def test_nested_fuzz(dev, kernel, seed):
    rng = np.random.default_rng(500 + seed)
    n = 2000
    w = workload.nested(n, seed=seed)
    stream, ends = O.encode_nested_batch(w)
    recs = [bytes(stream[(int(ends[i - 1]) if i else 0):int(ends[i])]) for i in range(n)]
    out = []
    for r in recs:
        b = bytearray(r)
        x = rng.integers(0, 5)
        if x == 0:
            for _ in range(rng.integers(1, 4)):
                b[rng.integers(0, len(b))] = rng.integers(0, 256)
        elif x == 1:
            b = b[rng.integers(0, len(b)):]
        elif x == 2:
            b = b[:rng.integers(0, len(b))]
        out.append(bytes(b))
    s2, e2 = concat_records(out)
    check_nested(dev, s2, e2, f"fuzz {seed}")


def nested_device_inputs(w, dev):
    """workload.nested arrays -> (outer_cols, outer_heaps, item_begin, item_cols, item_heaps) on dev."""
    n = len(w["seq"])
    outer = [to_dev(w["id"], dev), to_dev(w["seq"].view(np.uint8).reshape(n, 8), dev),
             to_dev(w["name"].view(np.uint8).reshape(n, 8), dev), None]
    m = len(w["key"])
    items = [to_dev(w["key"].view(np.uint8).reshape(m, 4), dev), to_dev(w["value"].view(np.uint8).reshape(m, 8), dev),
             to_dev(w["label"].view(np.uint8).reshape(m, 8), dev)]
    return (outer, {2: to_dev(w["name_heap"], dev)}, to_dev(w["item_begin"].view(np.int32), dev), items,
            {2: to_dev(w["label_heap"] if w["label_heap"].size else np.zeros(1, np.uint8), dev)})


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 5000])
def test_nested_encode_bitexact(dev, kernel, n):
    import torch

    w = workload.nested(n, seed=n + 3)
    want, want_ends = O.encode_nested_batch(w)
    oc, oh, ib, ic, ih = nested_device_inputs(w, dev)
    out, ends = spec_amd.encode_nested(NESTED, oc, oh, ib, ic, ih, n)
    torch.cuda.synchronize()
    assert np.array_equal(ends.cpu().numpy().view(np.uint64), want_ends)
    assert np.array_equal(out.cpu().numpy(), want)


@pytest.mark.parametrize("n", [1, 100, 5000])
def test_nested_encode_workspace_sizes(dev, kernel, n):
    """The same bytes with the minimal workspace (spec_encode_nested_workspace_size: the write pass
    recomputes the item prefixes) and the larger one (..._size_items: it reads the size pass's)."""
    import ctypes as C

    import torch

    from spec_amd import _lib

    w = workload.nested(n, seed=n + 11, count=(0, 12))
    want, want_ends = O.encode_nested_batch(w)
    oc, oh, ib, ic, ih = nested_device_inputs(w, dev)
    m = int(ic[0].shape[0])
    L = _lib.lib()
    for ws in (L.spec_encode_nested_workspace_size(n), L.spec_encode_nested_workspace_size_items(n, m)):
        enc = spec_amd.NestedEncoder(NESTED, n, dev)
        enc.workspace = torch.empty((ws + 7) // 8, dtype=torch.int64, device=dev)
        enc.ws_bytes = ws
        out = torch.empty(len(want), dtype=torch.uint8, device=dev)
        ends = torch.empty(n, dtype=torch.int64, device=dev)
        rc = L.spec_encode_nested(
            C.byref(NESTED.c), enc._ptrs(oc), *enc._heaps(NESTED.outer.fields, oh), C.c_void_p(ib.data_ptr()),
            enc._ptrs(ic), *enc._heaps(NESTED.item.fields, ih), m, n, C.c_void_p(out.data_ptr()), out.numel(),
            C.c_void_p(ends.data_ptr()), C.c_void_p(enc.workspace.data_ptr()), ws, C.c_void_p(enc.total.data_ptr()),
            None)
        assert rc == 0
        torch.cuda.synchronize()
        assert np.array_equal(ends.cpu().numpy().view(np.uint64), want_ends), ws
        assert np.array_equal(out.cpu().numpy(), want), ws


def test_nested_encode_big_lists_and_empty(dev, kernel):
    """Lists of 0 and > 255 items (IsBigList by count), long labels (big items / big lists by
    offset), in one batch."""
    import torch

    w = workload.nested(300, seed=9, count=(0, 3))
    counts = np.diff(w["item_begin"]).astype(np.int64)
    counts[5] = 300
    counts[7] = 0
    counts[11] = 2
    rng = np.random.default_rng(1)
    m = int(counts.sum())
    ib = np.zeros(len(counts) + 1, np.uint32)
    np.cumsum(counts, out=ib[1:])
    lens = rng.integers(0, 12, m).astype(np.uint32)
    lens[ib[11]] = 70000  # one big item (data > 65535) => big item table, big list by offset
    label = np.zeros((m, 2), np.uint32)
    label[1:, 0] = np.cumsum(lens[:-1])
    label[:, 1] = lens
    w.update(item_begin=ib, key=rng.integers(-2**31, 2**31, m).astype(np.int32),
             value=rng.standard_normal(m), label=label,
             label_heap=rng.integers(32, 127, int(lens.sum()), dtype=np.uint8))
    want, want_ends = O.encode_nested_batch(w)
    oc, oh, ibd, ic, ih = nested_device_inputs(w, dev)
    out, ends = spec_amd.encode_nested(NESTED, oc, oh, ibd, ic, ih, 300)
    torch.cuda.synchronize()
    assert np.array_equal(ends.cpu().numpy().view(np.uint64), want_ends)
    assert np.array_equal(out.cpu().numpy(), want)
    check_nested(dev, want, want_ends, "big lists decode")


def test_nested_roundtrip_full_size(dev):
    """config 4 at 1M records: GPU encode == oracle bytes, and GPU decode of them == inputs."""
    import torch

    n = 1 << 20
    w = workload.nested(n)
    want, want_ends = O.encode_nested_batch(w)
    oc, oh, ib, ic, ih = nested_device_inputs(w, dev)
    out, ends = spec_amd.encode_nested(NESTED, oc, oh, ib, ic, ih, n)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    m = len(w["key"])
    for onepass in (False, True):
        got = spec_amd.decode_nested(NESTED, out, ends, onepass=onepass)
        assert int(got.status.sum()) == 0
        assert got.total_items == m
        assert np.array_equal(got.item_begin.cpu().numpy().view(np.uint32), w["item_begin"])
        assert np.array_equal(got.items[0][:m].cpu().numpy().view(np.int32).ravel(), w["key"])
        assert np.array_equal(got.items[1][:m].cpu().numpy().view(np.uint64).ravel(), w["value"].view(np.uint64))
        assert int(got.item_status[:m].sum()) == 0
        assert np.array_equal(got.outer[1].cpu().numpy().view(np.int64).ravel(), w["seq"])


def test_nested_encode_many_items_per_wave(dev, kernel):
    """Waves owning more than NENC_ITEM_CAP (512) items take the per-lane path; neighbours
    with fewer items take the item-parallel path — one batch, both paths."""
    import torch

    n = 640
    w = workload.nested(n, seed=21, count=(0, 6))
    counts = np.diff(w["item_begin"]).astype(np.int64)
    counts[128:192] = 12  # 768 items in the third wave
    rng = np.random.default_rng(5)
    m = int(counts.sum())
    ib = np.zeros(n + 1, np.uint32)
    np.cumsum(counts, out=ib[1:])
    lens = rng.integers(0, 12, m).astype(np.uint32)
    label = np.zeros((m, 2), np.uint32)
    label[1:, 0] = np.cumsum(lens[:-1])
    label[:, 1] = lens
    w.update(item_begin=ib, key=rng.integers(-2**31, 2**31, m).astype(np.int32),
             value=rng.standard_normal(m), label=label,
             label_heap=rng.integers(32, 127, int(lens.sum()), dtype=np.uint8))
    want, want_ends = O.encode_nested_batch(w)
    oc, oh, ibd, ic, ih = nested_device_inputs(w, dev)
    out, ends = spec_amd.encode_nested(NESTED, oc, oh, ibd, ic, ih, n)
    torch.cuda.synchronize()
    assert np.array_equal(ends.cpu().numpy().view(np.uint64), want_ends)
    assert np.array_equal(out.cpu().numpy(), want)


# A schema unlike NESTED: the list is the FIRST outer field (items start right at the record
# start, so an item's head store lands in the previous record's bytes), item tags > 255 (big
# item tables) and a repeated item tag (Writer tie order).
GEN_OUTER = [(7, Kind.LIST), (2, Kind.BYTE), (9, Kind.STRING), (3, Kind.UINT32)]
GEN_ITEM = [(4, Kind.BOOL), (1, Kind.UINT16), (300, Kind.BIN64), (2, Kind.BYTES), (1, Kind.INT16)]


def _spans(rng, lens):
    sp = np.zeros((len(lens), 2), np.uint32)
    if len(lens):
        sp[1:, 0] = np.cumsum(lens[:-1])
    sp[:, 1] = lens
    return sp, rng.integers(32, 127, int(np.sum(lens)), dtype=np.uint8)


def _writer_encode_generic(c):
    """The oracle Writer, record by record, for GEN_OUTER/GEN_ITEM (pure Python loop)."""
    recs = []
    ib = c["item_begin"]
    for r in range(len(c["byte"])):
        wr = O.Writer()
        wr.message()
        wr.field_list(7)
        for i in range(int(ib[r]), int(ib[r + 1])):
            wr.elem_message()
            wr.field(4, "bool", int(c["bool"][i]))
            wr.field(1, "uint16", int(c["u16"][i]))
            wr.field(300, "bin64", c["bin"][i].tobytes())
            o, ln = c["bytes"][i]
            wr.field(2, "bytes", c["bytes_heap"][o:o + ln].tobytes())
            wr.field(1, "int16", int(c["i16"][i]))
            assert wr.end()[1] is None
        assert wr.end()[1] is None
        wr.field(2, "byte", int(c["byte"][r]))
        o, ln = c["str"][r]
        wr.field(9, "string", c["str_heap"][o:o + ln].tobytes())
        wr.field(3, "uint32", int(c["u32"][r]))
        b, err = wr.end()
        assert err is None, err
        recs.append(b)
        wr.close()
    return concat_records(recs)


def test_nested_encode_generic_schema(dev, kernel):
    import torch

    schema = spec_amd.NestedSchema(GEN_OUTER, GEN_ITEM)
    rng = np.random.default_rng(77)
    n = 700
    counts = rng.integers(0, 7, n)
    counts[200:264] = 10        # a wave over the item cap (per-lane path)
    counts[3] = 300             # a big list by count
    slen = rng.integers(0, 30, n).astype(np.uint32)
    slen[500] = 20000           # a wave whose output does not fit the LDS slab
    ib = np.zeros(n + 1, np.uint32)
    np.cumsum(counts, out=ib[1:])
    m = int(ib[-1])
    blen = rng.integers(0, 9, m).astype(np.uint32)
    c = {"item_begin": ib, "byte": rng.integers(0, 256, n, dtype=np.uint8),
         "u32": rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) >> rng.integers(0, 32, n).astype(np.uint32),
         "bool": rng.integers(0, 2, m, dtype=np.uint8), "u16": rng.integers(0, 2**16, m).astype(np.uint16),
         "bin": rng.integers(0, 256, (m, 8), dtype=np.uint8),
         "i16": rng.integers(-2**15, 2**15, m).astype(np.int16)}
    c["str"], c["str_heap"] = _spans(rng, slen)
    c["bytes"], c["bytes_heap"] = _spans(rng, blen)
    want, want_ends = _writer_encode_generic(c)
    outer = [None, to_dev(c["byte"], dev), to_dev(c["str"], dev), to_dev(c["u32"], dev)]
    items = [to_dev(c["bool"], dev), to_dev(c["u16"], dev), to_dev(c["bin"], dev), to_dev(c["bytes"], dev),
             to_dev(c["i16"], dev)]
    out, ends = spec_amd.encode_nested(schema, outer, {2: to_dev(c["str_heap"], dev)}, to_dev(ib.view(np.int32), dev),
                                       items, {3: to_dev(c["bytes_heap"], dev)}, n)
    torch.cuda.synchronize()
    assert np.array_equal(ends.cpu().numpy().view(np.uint64), want_ends)
    assert np.array_equal(out.cpu().numpy(), want)


def test_nested_encode_errors(dev, kernel):
    """An item string outside its heap or a non-monotonic item_begin is an encoder error."""
    n = 300
    w = workload.nested(n, seed=4)
    oc, oh, ib, ic, ih = nested_device_inputs(w, dev)
    bad = w["label"].copy()
    bad[len(bad) // 2, 1] = 1 << 20
    with pytest.raises(spec_amd.SpecError):
        spec_amd.encode_nested(NESTED, oc, oh, ib, [ic[0], ic[1], to_dev(bad, dev)], ih, n)
    ib2 = w["item_begin"].copy()
    ib2[100] = ib2[102] + 1
    with pytest.raises(spec_amd.SpecError):
        spec_amd.encode_nested(NESTED, oc, oh, to_dev(ib2.view(np.int32), dev), ic, ih, n)


# ---- nested schemas with a half of more than 64 fields (round 5) --------------------------------
# Decoded in chunks of 64 fields per half (the run-time kernels), encoded through the schema-tree
# encoder; the oracle is the tree oracle over the equivalent tree (a record message whose list
# field is a list of item messages: the same Writer calls, writer_list_msg.go:8-47).

_WK = [Kind.BOOL, Kind.BYTE, Kind.INT16, Kind.INT32, Kind.INT64, Kind.UINT16, Kind.UINT32, Kind.UINT64,
       Kind.FLOAT32, Kind.FLOAT64, Kind.BIN64, Kind.BIN128, Kind.STRING, Kind.BYTES]


def _wide_nested(no=70, ni=80, list_at=30):
    from spec_amd.tree import ListOf, Message, Tree

    outer = [(i + 1, _WK[i % len(_WK)]) for i in range(no)]
    outer[list_at] = (list_at + 1, Kind.LIST)
    outer[5] = (400, outer[5][1])  # a tag past 255: big record tables
    item = [(j + 1, _WK[(3 * j + 1) % len(_WK)]) for j in range(ni)]
    schema = spec_amd.NestedSchema(outer, item)
    imsg = Message("Item", [(f"w{j}", t, k) for j, (t, k) in enumerate(item)])
    tree = Tree(Message("Outer", [(f"o{i}", t, ListOf(imsg) if k == Kind.LIST else k) for i, (t, k) in enumerate(outer)]))
    return schema, tree, list_at


def _wide_inputs(tree, schema, list_at, n, seed, dev):
    from tests.tree_helpers import oracle_encode

    cols, heaps, rows = workload.tree_batch(tree, n, seed, count=(0, 4))
    lp = f"o{list_at}"
    cols[f"{lp}?"] = np.ones_like(cols[f"{lp}?"])  # a nested list is always written
    rows = [n, int(cols[f"{lp}#begin"].view(np.uint32).reshape(-1)[n])]
    want_stream, want_ends = oracle_encode(tree, cols, heaps, n)
    outer = [None if k == Kind.LIST else to_dev(cols[f"o{i}"], dev) for i, k in enumerate(f.kind for f in schema.outer.fields)]
    oh = {i: to_dev(heaps[f"o{i}"], dev) for i, k in enumerate(f.kind for f in schema.outer.fields)
          if k in (Kind.STRING, Kind.BYTES)}
    items = [to_dev(cols[f"{lp}[].w{j}"], dev) for j in range(len(schema.item.fields))]
    ih = {j: to_dev(heaps[f"{lp}[].w{j}"], dev) for j, k in enumerate(f.kind for f in schema.item.fields)
          if k in (Kind.STRING, Kind.BYTES)}
    ib = to_dev(cols[f"{lp}#begin"].view(np.uint32).reshape(-1).view(np.int32), dev)
    return cols, heaps, rows, want_stream, want_ends, outer, oh, items, ih, ib


@pytest.mark.parametrize("n", [1, 700])
def test_nested_wide_encode_decode(dev, n):
    """Halves of 70 (a big-tag table, the list in the middle) and 80 fields: encoded bytes and
    ends bit-exact against the tree oracle; decoded (index + chunked decode, and one pass) outer
    and item columns identical to the tree oracle's VALUE columns, item_begin = its BEGIN."""
    import torch

    from tests.tree_helpers import oracle_decode

    schema, tree, list_at = _wide_nested()
    cols, heaps, rows, ws, we, outer, oh, items, ih, ib = _wide_inputs(tree, schema, list_at, n, 900 + n, dev)
    out, ends = spec_amd.encode_nested(schema, outer, oh, ib, items, ih, n)
    torch.cuda.synchronize()
    assert np.array_equal(ends.cpu().numpy().view(np.uint64), we)
    assert np.array_equal(out.cpu().numpy(), ws)
    wrows, want = oracle_decode(tree, ws, we)
    wcol = {c.name: w for c, w in zip(tree.columns, want)}
    d_s, d_e = to_dev(ws, dev), to_dev(we.view(np.int64), dev)
    for onepass in (False, True):
        got = spec_amd.decode_nested(schema, d_s, d_e, onepass=onepass)
        torch.cuda.synchronize()
        assert got.total_items == wrows[1]
        assert np.array_equal(got.item_begin.cpu().numpy().view(np.uint32), wcol[f"o{list_at}#begin"].view(np.uint32).reshape(-1))
        assert not got.status.cpu().numpy().any()
        for i, k in enumerate(f.kind for f in schema.outer.fields):
            if k == Kind.LIST:
                continue
            g = got.outer[i].cpu().numpy()
            w = wcol[f"o{i}"].reshape(g.shape)
            if k in (Kind.STRING, Kind.BYTES):  # spans: same stream, same offsets
                assert np.array_equal(g, w), (onepass, i)
            else:
                assert np.array_equal(g, w), (onepass, i)
        for j in range(len(schema.item.fields)):
            g = got.items[j].cpu().numpy()[: wrows[1]]
            assert np.array_equal(g, wcol[f"o{list_at}[].w{j}"].reshape(g.shape)), (onepass, j)


def test_nested_wide_encode_errors(dev):
    """A wide nested schema's encoder errors: an item string outside its heap, item_begin not
    monotonic (*total all-ones: spec_encode_nested raises)."""
    schema, tree, list_at = _wide_nested()
    n = 200
    cols, heaps, rows, ws, we, outer, oh, items, ih, ib = _wide_inputs(tree, schema, list_at, n, 950, dev)
    j = next(j for j, k in enumerate(f.kind for f in schema.item.fields) if k == Kind.STRING)
    bad = cols[f"o{list_at}[].w{j}"].copy()
    bad.view(np.uint32).reshape(-1, 2)[len(bad) // 2, 1] = 1 << 24
    items2 = list(items)
    items2[j] = to_dev(bad, dev)
    with pytest.raises(spec_amd.SpecError):
        spec_amd.encode_nested(schema, outer, oh, ib, items2, ih, n)
    b2 = cols[f"o{list_at}#begin"].view(np.uint32).reshape(-1).copy()
    b2[100] = b2[102] + 1
    with pytest.raises(spec_amd.SpecError):
        spec_amd.encode_nested(schema, outer, oh, to_dev(b2.view(np.int32), dev), items, ih, n)
