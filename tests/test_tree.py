"""Schema trees on the CPU: the engine's layout (spec_tree_layout, host code) against the
oracle's restatement, the oracle's generated-reader/-writer restatement (oracle/tree.c) against
the reference's own test object (internal/tests/pkg1/test.go + pkg1_test.go) and known bytes,
and oracle round trips of random trees."""
from __future__ import annotations

import ctypes as C
import struct

import numpy as np
import pytest

import spec_amd
from oracle import oracle as O
from spec_amd import Kind, ListOf, Message, Struct, Tree, workload
from tests.trees import many_tables_tree, wide_tree
from tests.tree_helpers import oracle_decode, oracle_encode, oracle_fields, roundtrip_mismatches, shapes_tree


def _layout_equal(tree: Tree):
    want = O.tree_layout(oracle_fields(tree))
    assert want is not None
    tables, cols = want
    assert len(tables) == len(tree.tables) and len(cols) == len(tree.columns)
    for t, w in zip(tree.tables, tables):
        assert (t.parent, t.field, t.rel, t.shape) == (w["parent"], w["field"], w["rel"], w["shape"]), t.path
        assert (t.columns[0].index, len(t.columns)) == (w["first_column"], w["ncolumns"]), t.path
    for c, w in zip(tree.columns, cols):
        assert (c.table, c.field, c.role, c.kind, c.width) == (w["table"], w["field"], w["role"], w["kind"], w["width"]), c.name


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_layout_matches_oracle_pkg1(depth):
    _layout_equal(spec_amd.pkg1_tree(depth))


def test_layout_matches_oracle_shapes():
    _layout_equal(shapes_tree())


def test_invalid_trees_rejected_by_both():
    bad = [
        [(1, Kind.INT32, 0, 0)],                                    # parent not earlier
        [(1, Kind.STRUCT, 0, -1), (0, Kind.MESSAGE, 0, 0)],         # message inside a struct
        [(1, Kind.LIST, Kind.INT64, -1), (1, Kind.INT32, 0, 0)],    # child of a scalar list
        [(1, Kind.INT32, 0, -1), (1, Kind.INT32, 0, 0)],            # child of a scalar
        [(1, 33, 0, -1)],                                           # unknown kind
        [(1, Kind.LIST, Kind.ANY, -1)],                             # list of any
    ]
    L = spec_amd.lib()
    for fields in bad:
        assert O.tree_layout(O.tree_fields(fields)) is None, fields
        t = spec_amd._lib.SpecTree()
        t.nfields = len(fields)
        for i, (tag, kind, elem, parent) in enumerate(fields):
            t.fields[i].tag, t.fields[i].kind, t.fields[i].elem, t.fields[i].parent = tag, kind, elem, parent
        nt, nc = C.c_uint32(), C.c_uint32()
        assert L.spec_tree_layout(C.byref(t), None, C.byref(nt), None, C.byref(nc)) == -1, fields


def test_struct_known_bytes():
    """Struct{key 1, value -1} as pkg1 TestStruct: members through their encoders then
    EncodeStruct (internal/encode/struct.go:14-21): int32 1 = zigzag 2, -1 = zigzag 1."""
    tree = Tree(Message("M", [("s", 61, Struct("Struct", [("key", Kind.INT32), ("value", Kind.INT32)]))]))
    cols = {"s.key": np.array([[1, 0, 0, 0]], np.uint8), "s.value": np.full((1, 4), 0xff, np.uint8),
            "#status": np.zeros((1, 1), np.uint8)}
    stream, ends = oracle_encode(tree, cols, {}, 1)
    struct_bytes = bytes([0x02, 0x0B, 0x01, 0x0B, 0x04, 0x5A])
    # message: data | table (tag 61, end 6) | dataSize 6 | tableSize 3 | TypeMessage
    assert bytes(stream) == struct_bytes + bytes([61, 0, 6, 6, 3, 0x50])
    rows, got = oracle_decode(tree, stream, ends)
    assert rows == [1] and got[0].view(np.int32)[0, 0] == 1 and got[1].view(np.int32)[0, 0] == -1


def test_value_list_known_bytes():
    """ints = [0, 1, 2]: elements int64 (zigzag 0, 2, 4), list table of u16 BE end offsets
    (internal/encode/list.go:15-75)."""
    tree = Tree(Message("M", [("ints", 70, ListOf(Kind.INT64))]))
    cols = {"ints?": np.ones((1, 1), np.uint8), "ints#begin": np.array([0, 3], np.uint32).view(np.uint8).reshape(2, 4),
            "ints[]": np.array([0, 1, 2], np.int64).view(np.uint8).reshape(3, 8)}
    stream, ends = oracle_encode(tree, cols, {}, 1)
    lst = bytes([0x00, 0x0C, 0x02, 0x0C, 0x04, 0x0C, 0, 2, 0, 4, 0, 6, 6, 6, 0x46])
    assert bytes(stream) == lst + bytes([70, 0, len(lst), len(lst), 3, 0x50])
    rows, got = oracle_decode(tree, stream, ends)
    g = {c.name: v for c, v in zip(tree.columns, got)}
    assert rows == [1, 3] and list(g["ints[]"].view(np.int64).ravel()) == [0, 1, 2]


def _test_object_columns(tree: Tree):
    """pkg1.TestObject (internal/tests/pkg1/test.go:16-110) as one record of columns."""
    def c(v):
        return np.ascontiguousarray(np.atleast_1d(v)).view(np.uint8).reshape(len(np.atleast_1d(v)), -1)

    heaps, cols = {}, {}

    def strings(name, vals):
        data = b"".join(v.encode() for v in vals)
        offs = np.cumsum([0] + [len(v) for v in vals])[:-1]
        heaps[name] = np.frombuffer(data or b"\0", np.uint8).copy()
        cols[name] = np.stack([offs, [len(v) for v in vals]], 1).astype(np.uint32).view(np.uint8)

    bin64 = np.zeros(8, np.uint8); bin64[7] = 1                     # bin.Int64(1)
    bin128 = np.zeros(16, np.uint8); bin128[15] = 2                 # bin.Int128(0, 2)
    bin256 = np.zeros(32, np.uint8); bin256[31] = 3                 # bin.Int256(0, 0, 0, 3)
    cols.update({
        "bool": c(np.uint8(1)), "byte": c(np.uint8(255)), "int16": c(np.int16(32767)), "int32": c(np.int32(2**31 - 1)),
        "int64": c(np.int64(2**63 - 1)), "uint16": c(np.uint16(65535)), "uint32": c(np.uint32(2**32 - 1)),
        "uint64": c(np.uint64(2**64 - 1)), "float32": c(np.float32(3.4028234663852886e38)),
        "float64": c(np.float64(1.7976931348623157e308)), "bin64": bin64.reshape(1, 8), "bin128": bin128.reshape(1, 16),
        "bin256": bin256.reshape(1, 32), "enum1": c(np.int32(1)), "struct1.key": c(np.int32(1)),
        "struct1.value": c(np.int32(-1)), "message1.f1": c(np.int32(1)), "message1.f2": c(np.int32(2)),
        "message1.f3": c(np.int32(3)),
    })
    strings("string", ["hello, world"])
    strings("bytes1", ["goodbye, world"])
    strings("submessage.value", ["value 000"])
    strings("submessage.next.value", [""])
    strings("submessage1.key", ["key 000"])
    cols["submessage1.value.x"] = c(np.int32(0))
    cols["submessage1.value.y"] = c(np.int32(0))
    for p in ("message1?", "submessage?", "submessage1?", "ints?", "strings?", "structs?", "submessages?", "submessages1?"):
        cols[p] = np.ones((1, 1), np.uint8)
    cols["submessage.next?"] = np.zeros((1, 1), np.uint8)
    ten = np.array([0, 10], np.uint32).view(np.uint8).reshape(2, 4)
    for l in ("ints", "strings", "structs", "submessages", "submessages1"):
        cols[f"{l}#begin"] = ten
    cols["ints[]"] = c(np.arange(10, dtype=np.int64))
    strings("strings[]", [f"hello, world {i:03d}" for i in range(10)])
    cols["structs[].key"] = c(np.arange(10, dtype=np.int32))
    cols["structs[].value"] = c(-np.arange(10, dtype=np.int32))
    strings("submessages[].value", [f"value {i:03d}" for i in range(10)])
    cols["submessages[].next?"] = np.zeros((10, 1), np.uint8)
    strings("submessages[].next.value", [""] * 10)
    strings("submessages1[].key", [f"key {i:03d}" for i in range(10)])
    cols["submessages1[].value.x"] = c(np.arange(10, dtype=np.int32))
    cols["submessages1[].value.y"] = c(-np.arange(10, dtype=np.int32))
    anyb = struct.pack(">d", 2.5) + bytes([41])
    heaps["any"] = np.frombuffer(anyb, np.uint8).copy()
    cols["any"] = np.array([[0, len(anyb)]], np.uint32).view(np.uint8)
    for t in tree.tables:
        cols.setdefault(f"{t.path}#status", None)
    rows = [1] * len(tree.tables)
    for t in tree.tables:
        if t.rel == 2:
            rows[t.index] = 10
        elif t.rel == 1:
            rows[t.index] = rows[t.parent]
    for t in tree.tables:
        cols[f"{t.path}#status"] = np.zeros((rows[t.index], 1), np.uint8)
    return cols, heaps


def test_oracle_test_object_roundtrip():
    """What pkg1_test.go asserts through the generated getters, on the oracle restatement: every
    scalar at its extreme, struct1 {1, -1}, the sub-messages, and the 10-element lists."""
    tree = spec_amd.pkg1_tree()
    cols, heaps = _test_object_columns(tree)
    stream, ends = oracle_encode(tree, cols, heaps, 1)
    # the record parses (ParseMessage: recursive validation consumes the whole buffer)
    st, sz = O.parse_batch(stream, ends)
    assert st[0] == 0 and sz[0] == len(stream)
    rows, got = oracle_decode(tree, stream, ends)
    g = {c.name: v for c, v in zip(tree.columns, got)}
    assert g["int64"].view(np.int64)[0, 0] == 2**63 - 1 and g["uint64"].view(np.uint64)[0, 0] == 2**64 - 1
    assert g["float32"].view(np.float32)[0, 0] == np.float32(3.4028234663852886e38)
    assert list(g["ints[]"].view(np.int64).ravel()) == list(range(10))
    assert list(g["structs[].value"].view(np.int32).ravel()) == [-i for i in range(10)]
    vals = g["submessages[].value"].view(np.uint32).reshape(-1, 2)
    assert [bytes(stream[o:o + n]).decode() for o, n in vals] == [f"value {i:03d}" for i in range(10)]
    assert g["submessages[].next?"].ravel().tolist() == [0] * 10 and g["submessage?"][0, 0] == 1
    anys = g["any"].view(np.uint32)[0]
    assert bytes(stream[anys[0]:anys[0] + anys[1]]) == bytes(heaps["any"])
    assert roundtrip_mismatches(tree, cols, heaps, got, stream) == []


@pytest.mark.parametrize("seed,n", [(1, 300), (2, 300), (3, 1), (4, 2)])
def test_oracle_roundtrip_random_pkg1(seed, n):
    tree = spec_amd.pkg1_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, seed)
    stream, ends = oracle_encode(tree, cols, heaps, n)
    st, _ = O.parse_batch(stream, ends)
    assert not st.any()
    got_rows, got = oracle_decode(tree, stream, ends)
    assert got_rows == rows
    assert roundtrip_mismatches(tree, cols, heaps, got, stream) == []


def test_oracle_roundtrip_shapes_big_lists():
    tree = shapes_tree()
    cols, heaps, rows = workload.tree_batch(tree, 40, 5, count=(0, 300))
    stream, ends = oracle_encode(tree, cols, heaps, 40)
    got_rows, got = oracle_decode(tree, stream, ends)
    assert got_rows == rows and max(rows) > 255
    assert roundtrip_mismatches(tree, cols, heaps, got, stream) == []


def test_oracle_struct_reverse_decode_partial():
    """Generated struct Decode reads members from the last; an error stops it with the members
    already decoded kept (internal/lang/generator/struct.go:83-107): a struct whose FIRST member
    is corrupt still yields its second."""
    tree = Tree(Message("M", [("s", 1, Struct("S", [("a", Kind.INT32), ("b", Kind.INT32)]))]))
    body = bytes([0x02, 0x33]) + bytes([0x04, 0x0B])  # a: type 0x33 (no such type), b = int32 2
    val = body + bytes([len(body), 0x5A])
    rec = val + bytes([1, 0, len(val), len(val), 3, 0x50])
    rows, got = oracle_decode(tree, np.frombuffer(rec, np.uint8), np.array([len(rec)], np.uint64))
    assert got[1].view(np.int32)[0, 0] == 2 and got[0].view(np.int32)[0, 0] == 0


# ---- structs inside structs (internal/lang/model/struct_field.go:57-70) ----

def _nested_tree():
    from tests.tree_helpers import nested_struct_tree

    return nested_struct_tree()


def test_layout_matches_oracle_nested_structs():
    tree = _nested_tree()
    _layout_equal(tree)
    # inner structs' members sit in place, pre-order, with dotted names
    names = [c.name for c in tree.tables[0].columns]
    assert names[:6] == ["id", "outer.a", "outer.in.x", "outer.in.y", "outer.s", "outers?"]
    assert "deep.m.j.y" in names and "deep.o.in.x" in names
    assert [c.name for c in tree.tables[1].columns][:4] == ["outers#begin", "outers[].a", "outers[].in.x", "outers[].in.y"]


def test_nested_struct_known_bytes():
    """Outer{a 1, in Inner{x -1, y "hi"}, s ""}: the inner struct is Inner's own EncodeInnerTo
    (members, then EncodeStruct) inside Outer's data (generator/struct.go:115-142)."""
    inner = Struct("Inner", [("x", Kind.INT32), ("y", Kind.STRING)])
    tree = Tree(Message("M", [("o", 1, Struct("Outer", [("a", Kind.INT32), ("in", inner), ("s", Kind.STRING)]))]))
    heaps = {"o.in.y": np.frombuffer(b"hi", np.uint8).copy(), "o.s": np.zeros(1, np.uint8)}
    cols = {"o.a": np.array([[1, 0, 0, 0]], np.uint8), "o.in.x": np.full((1, 4), 0xff, np.uint8),
            "o.in.y": np.array([[0, 2]], np.uint32).view(np.uint8), "o.s": np.zeros((1, 8), np.uint8),
            "#status": np.zeros((1, 1), np.uint8)}
    stream, ends = oracle_encode(tree, cols, heaps, 1)
    inner_b = bytes([0x01, 0x0B]) + b"hi" + bytes([0x00, 0x02, 0x3C])
    inner_b += bytes([len(inner_b), 0x5A])
    outer_data = bytes([0x02, 0x0B]) + inner_b + bytes([0x00, 0x00, 0x3C])
    outer_b = outer_data + bytes([len(outer_data), 0x5A])
    assert bytes(stream) == outer_b + bytes([1, 0, len(outer_b), len(outer_b), 3, 0x50])
    rows, got = oracle_decode(tree, stream, ends)
    g = {c.name: v for c, v in zip(tree.columns, got)}
    assert g["o.a"].view(np.int32)[0, 0] == 1 and g["o.in.x"].view(np.int32)[0, 0] == -1
    off, ln = g["o.in.y"].view(np.uint32)[0]
    assert bytes(stream[off:off + ln]) == b"hi" and g["#status"][0, 0] == 0


def test_nested_struct_reverse_decode_partial():
    """An inner struct's Decode errs: the outer stops there; members decoded before (the ones
    after it in declaration order) keep their values, and the inner struct keeps what it decoded
    (generator/struct.go:83-107 at both levels)."""
    inner = Struct("Inner", [("x", Kind.INT32), ("y", Kind.INT32)])
    tree = Tree(Message("M", [("o", 1, Struct("Outer", [("a", Kind.INT32), ("in", inner), ("s", Kind.INT32)]))]))
    ib = bytes([0x02, 0x33]) + bytes([0x06, 0x0B])   # x: bad type, y = 3
    ib += bytes([len(ib), 0x5A])
    ob = bytes([0x04, 0x0B]) + ib + bytes([0x08, 0x0B])  # a = 2, in, s = 4
    ob += bytes([len(ob), 0x5A])
    rec = ob + bytes([1, 0, len(ob), len(ob), 3, 0x50])
    rows, got = oracle_decode(tree, np.frombuffer(rec, np.uint8), np.array([len(rec)], np.uint64))
    g = {c.name: v.view(np.int32)[0, 0] for c, v in zip(tree.columns, got) if c.name.startswith("o.")}
    assert g == {"o.a": 0, "o.in.x": 0, "o.in.y": 3, "o.s": 4}


@pytest.mark.parametrize("seed,n", [(1, 200), (2, 1), (3, 57)])
def test_oracle_roundtrip_nested_structs(seed, n):
    tree = _nested_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, seed)
    stream, ends = oracle_encode(tree, cols, heaps, n)
    st, _ = O.parse_batch(stream, ends)
    assert not st.any()
    got_rows, got = oracle_decode(tree, stream, ends)
    assert got_rows == rows
    assert roundtrip_mismatches(tree, cols, heaps, got, stream) == []


def test_struct_depth_limit():
    """At most 16 structs deep (SPEC_TREE_MAX_STRUCT_DEPTH); both the engine and the oracle
    reject a 17th level."""
    def chain(levels):
        s = Struct("L0", [("v", Kind.INT32)])
        for k in range(1, levels):
            s = Struct(f"L{k}", [("s", s), ("v", Kind.INT32)])
        return Message("M", [("s", 1, s)])

    t16 = Tree(chain(16))
    _layout_equal(t16)
    with pytest.raises(spec_amd.SpecError):
        Tree(chain(17))
    assert O.tree_layout(O.tree_fields([(1, Kind.STRUCT, 0, -1)] + [(0, Kind.STRUCT, 0, i) for i in range(16)]
                                       + [(0, Kind.INT32, 0, 16)])) is None


def test_specfile_nested_struct():
    from spec_amd import specfile

    sf = specfile.SpecSet()
    sf.add(specfile.load("""
        message M { o Outer 1; l []Outer 2; }
        struct Outer { a int32; in Inner; e Color; }
        struct Inner { x int64; y string; }
        enum Color { RED = 0; }
    """, "p"))
    tree = sf.tree("M", "p")
    names = [c.name for c in tree.columns]
    assert "o.in.x" in names and "l[].in.y" in names and "o.e" in names
    bad = specfile.SpecSet()
    bad.add(specfile.load("message M { o A 1; } struct A { b B; } struct B { a A; }", "q"))
    with pytest.raises(ValueError):
        bad.tree("M", "q")


def test_oracle_errmask_and_type():
    """ERRMASK bits (the direct fields' *Err getters, write order) and Value.Type() of any: an
    int32 field holding a string errs; a bool never errs; an absent field never errs; a list
    field holding an int64 errs (ListErr); an any field's type is its value's last byte."""
    wr = O.Writer()
    wr.message()
    wr.field(1, "string", "not an int")  # read as int32 -> Int32Err
    wr.field(2, "bool", True)
    wr.field(4, "int64", 5)              # read as a list -> ListErr
    wr.field(5, "float64", 2.5)          # any: type 41
    b, err = wr.end()
    assert err is None
    tree = Tree(Message("M", [("a", 1, Kind.INT32), ("b", 2, Kind.BOOL), ("c", 3, Kind.INT64),
                              ("l", 4, ListOf(Kind.INT32)), ("v", 5, Kind.ANY)]))
    rows, got = oracle_decode(tree, np.frombuffer(b, np.uint8), np.array([len(b)], np.uint64))
    g = {c.name: v for c, v in zip(tree.columns, got)}
    assert int(g["#errmask"].view(np.uint64)[0, 0]) == 0b01001
    assert g["v#type"][0, 0] == 41 and g["#status"][0, 0] == 0


def test_layout_matches_oracle_wide():
    """More than 64 direct fields (a message of 130, a struct of 70 members, an 80-field
    sub-message and list item): the same layout, ERRMASK ceil(direct / 64) words wide."""
    tree = wide_tree()
    _layout_equal(tree)
    assert [(c.name, c.width) for c in tree.columns if c.role == spec_amd.tree.ROLE_ERRMASK] == [
        ("#errmask", 24), ("sub#errmask", 16), ("subs[]#errmask", 16)]


@pytest.mark.parametrize("seed,n", [(1, 60), (2, 1)])
def test_oracle_roundtrip_wide(seed, n):
    tree = wide_tree()
    cols, heaps, rows = workload.tree_batch(tree, n, seed)
    stream, ends = oracle_encode(tree, cols, heaps, n)
    st, _ = O.parse_batch(stream, ends)
    assert not st.any()
    got_rows, got = oracle_decode(tree, stream, ends)
    assert got_rows == rows
    assert roundtrip_mismatches(tree, cols, heaps, got, stream) == []


def test_layout_matches_oracle_many_tables():
    """114 tables (100 sub-messages of the record, a list of items with 12 each) and a struct
    chain 14 deep: the same layout as the oracle's, and an oracle round trip."""
    tree = many_tables_tree()
    assert len(tree.tables) == 114
    _layout_equal(tree)
    cols, heaps, rows = workload.tree_batch(tree, 40, 3, count=(0, 3))
    stream, ends = oracle_encode(tree, cols, heaps, 40)
    got_rows, got = oracle_decode(tree, stream, ends)
    assert got_rows == rows
    assert roundtrip_mismatches(tree, cols, heaps, got, stream) == []


def test_oracle_errmask_words():
    """ERRMASK past 64 direct fields: the k-th field's *Err bit is bit k % 64 of word k / 64 —
    fields 0 and 66 of a 70-field message hold strings where int32s are read."""
    wr = O.Writer()
    wr.message()
    for i in range(70):
        if i in (0, 66):
            wr.field(i + 1, "string", "x")
        else:
            wr.field(i + 1, "int32", i)
    b, err = wr.end()
    assert err is None
    tree = Tree(Message("M", [(f"f{i}", i + 1, Kind.INT32) for i in range(70)]))
    rows, got = oracle_decode(tree, np.frombuffer(b, np.uint8), np.array([len(b)], np.uint64))
    g = {c.name: v for c, v in zip(tree.columns, got)}
    assert g["#errmask"].view(np.uint64)[0].tolist() == [1, 1 << 2]
    assert int(g["f65"].view(np.int32)[0, 0]) == 65


def test_oracle_spans_equal_records():
    """The oracle's decode over value spans (Field(tag).Message()) equals its decode over the same
    messages as contiguous records; a span past the stream is a panic row."""
    tree = spec_amd.pkg1_tree()
    cols, heaps, rows = workload.tree_batch(tree, 200, 12)
    stream, ends = oracle_encode(tree, cols, heaps, 200)
    starts = np.concatenate([[0], ends[:-1]])
    spans = np.stack([starts, ends - starts], 1).astype(np.uint32)
    r1, a = oracle_decode(tree, stream, ends)
    r2, b = O.decode_tree_spans(oracle_fields(tree), stream, spans)
    assert r1 == r2 and all(np.array_equal(x, y) for x, y in zip(a, b))
    spans[7] = (len(stream) - 1, 5)
    _, c = O.decode_tree_spans(oracle_fields(tree), stream, spans)
    st = {cc.name: v for cc, v in zip(tree.columns, c)}["#status"]
    assert st[7, 0] == 6 and not np.delete(st, 7).any()
