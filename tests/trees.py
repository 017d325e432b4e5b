"""Schema trees only the tests use (moved out of the product package): shapes the
GPU tests exercise beyond the reference's own .spec trees.  `extra_trees()` lists every tree whose
schema-specialised kernels build() precompiles for the tests; tests/make_precompile_list.py
writes them (with the product's trees) into the build-time list build() reads,
spec_amd/data/precompile_trees.json, and test_tree.py checks the list is current."""
from __future__ import annotations

from spec_amd.schema import Kind
from spec_amd.tree import ListOf, Message, Struct, Tree, pkg1_tree


def shapes_tree() -> Tree:
    """Lists inside list items, big tags (big message tables), value lists of every width, a
    struct with string members (pkg1.spec ComplexStruct), any."""
    complex_s = Struct("ComplexStruct", [("bin64", Kind.BIN64), ("bin128", Kind.BIN128), ("bin256", Kind.BIN256),
                                         ("string", Kind.STRING)])
    leaf = Message("Leaf", [("u", 1, Kind.UINT64), ("vals", 2, ListOf(Kind.INT16)), ("c", 3, complex_s)])
    item = Message("Item", [("name", 1, Kind.STRING), ("leaves", 2, ListOf(leaf)), ("f", 3, Kind.FLOAT32),
                            ("bytes", 4, ListOf(Kind.BYTES))])
    big = Message("Big", [("a", 300, Kind.INT32), ("b", 7, Kind.BOOL), ("any", 1000, Kind.ANY)])
    root = Message("Root", [
        ("id", 1, Kind.BIN128), ("items", 2, ListOf(item)), ("big", 3, big), ("u16s", 4, ListOf(Kind.UINT16)),
        ("f64s", 5, ListOf(Kind.FLOAT64)), ("bools", 6, ListOf(Kind.BOOL)), ("cs", 7, ListOf(complex_s)),
        ("seq", 65535, Kind.INT64),
    ])
    return Tree(root)


def nested_struct_tree() -> Tree:
    """Structs inside structs (internal/lang/model/struct_field.go:57-70): a struct field of a
    message, a list of such structs, a sub-message holding one, and three levels of nesting."""
    inner = Struct("Inner", [("x", Kind.INT32), ("y", Kind.STRING)])
    mid = Struct("Mid", [("i", inner), ("f", Kind.FLOAT64), ("j", inner)])
    outer = Struct("Outer", [("a", Kind.INT32), ("in", inner), ("s", Kind.STRING)])
    deep = Struct("Deep", [("m", mid), ("b", Kind.BIN64), ("o", outer)])
    sub = Message("Sub", [("o", 1, outer), ("n", 2, Kind.UINT16)])
    root = Message("Root", [
        ("id", 1, Kind.INT64), ("outer", 2, outer), ("outers", 3, ListOf(outer)), ("sub", 4, sub),
        ("deep", 5, deep), ("deeps", 6, ListOf(deep)), ("tail", 7, Kind.STRING),
    ])
    return Tree(root)


def wide_tree() -> Tree:
    """Messages and a struct with more than 64 direct fields (the reference's tables take any
    number of u16 tags: internal/format/msg.go:13-61): a record of 130 direct fields (scalars of
    every kind, tags past 255 making its table big, a 70-member struct, an 80-field sub-message,
    a list of them, any) — multi-word ERRMASK columns, the run-time decode group, generated
    writers over 100+ fields."""
    scalars = [Kind.BOOL, Kind.BYTE, Kind.INT16, Kind.INT32, Kind.INT64, Kind.UINT16, Kind.UINT32, Kind.UINT64,
               Kind.FLOAT32, Kind.FLOAT64, Kind.BIN64, Kind.BIN128, Kind.STRING, Kind.BYTES]
    wide = Message("Wide", [(f"w{i}", i + 1, scalars[(3 * i) % len(scalars)]) for i in range(80)])
    big_s = Struct("BigStruct", [(f"m{i}", scalars[(5 * i + 2) % len(scalars)]) for i in range(70)])
    fields = [(f"f{i}", (i + 1) if i % 40 != 39 else 300 + i, scalars[i % len(scalars)]) for i in range(126)]
    fields += [("st", 200, big_s), ("sub", 201, wide), ("subs", 202, ListOf(wide)), ("any", 203, Kind.ANY)]
    return Tree(Message("WideRoot", fields))


def many_tables_tree() -> Tree:
    """More than 64 tables and deep structs: a record with 100 sub-messages (one table each, all
    in the records' decode group: 100 range slots, so fewer waves per workgroup), a list of
    items holding 12 sub-messages each, and a struct chain 14 levels deep."""
    subs = [Message(f"S{i}", [("k", 1, Kind.INT32), ("s", 2, Kind.STRING)]) for i in range(100)]
    item_subs = [Message(f"T{i}", [("u", 1, Kind.UINT64), ("b", 2, Kind.BYTES)]) for i in range(12)]
    item = Message("Item", [("id", 1, Kind.INT64)] + [(f"t{i}", i + 2, m) for i, m in enumerate(item_subs)])
    deep = Struct("L0", [("v", Kind.INT32)])
    for k in range(1, 14):
        deep = Struct(f"L{k}", [("s", deep), ("v", Kind.INT16)])
    fields = [(f"s{i}", i + 1, m) for i, m in enumerate(subs)]
    fields += [("items", 101, ListOf(item)), ("deep", 102, deep), ("tail", 103, Kind.STRING)]
    return Tree(Message("ManyTables", fields))


def cross_kind_tree(shift: int) -> Tree:
    """pkg1's Message read with every scalar getter shifted to another kind
    (test_errmask_cross_kind's readers)."""
    fields = []
    for p, tag, k, e, par in pkg1_tree().to_fields():
        if 1 <= k <= 15:
            k = (k - 1 + shift) % 15 + 1
        fields.append((p, tag, k, e, par))
    return Tree.from_fields(fields)


def message1_tree() -> Tree:
    """Three int32 fields and a list of strings (test_gpu_tree's list-rows-outside-owner case)."""
    return Tree(Message("message1", [("f1", 1, Kind.INT32), ("f2", 2, Kind.INT32), ("f3", 3, Kind.INT32),
                                     ("l", 4, ListOf(Kind.STRING))]))


def extra_trees() -> dict:
    """{name: Tree} the GPU tests decode and encode beyond the product's own trees."""
    out = {"shapes": shapes_tree(), "nested_struct": nested_struct_tree(), "wide": wide_tree(),
           "many_tables": many_tables_tree(), "message1": message1_tree()}
    for shift in (1, 4, 9):
        out[f"cross_kind{shift}"] = cross_kind_tree(shift)
    return out
