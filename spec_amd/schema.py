"""Schema descriptors: which typed field each column holds.

A flat schema is the list of (tag, kind) a generated Write() emits in order — one
FieldWriter call per field (internal/lang/generator/message.go:319-439) — and that the
generated getters read back (message.go:97-186).  Kinds map one-to-one onto the typed
getters of types.Message (internal/types/msg.go:219-421).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass

import numpy as np

from ._lib import SPEC_MAX_FIELDS, SpecSchema


class Kind(enum.IntEnum):
    BOOL = 1
    BYTE = 2
    INT16 = 3
    INT32 = 4
    INT64 = 5
    UINT16 = 6
    UINT32 = 7
    UINT64 = 8
    FLOAT32 = 9
    FLOAT64 = 10
    BIN64 = 11
    BIN128 = 12
    BIN256 = 13
    STRING = 14
    BYTES = 15
    LIST = 16  # list<message> field of a NestedSchema's outer message (column = item_begin); tree lists
    STRUCT = 17   # spec_tree only
    MESSAGE = 18  # spec_tree only
    ANY = 19      # spec_tree only: a span of the raw value


WIDTH = {
    Kind.BOOL: 1, Kind.BYTE: 1, Kind.INT16: 2, Kind.INT32: 4, Kind.INT64: 8,
    Kind.UINT16: 2, Kind.UINT32: 4, Kind.UINT64: 8, Kind.FLOAT32: 4, Kind.FLOAT64: 8,
    Kind.BIN64: 8, Kind.BIN128: 16, Kind.BIN256: 32, Kind.STRING: 8, Kind.BYTES: 8,
    Kind.LIST: 0, Kind.STRUCT: 0, Kind.MESSAGE: 0, Kind.ANY: 8,
}

# numpy view of one column element (bins stay raw bytes)
NP_DTYPE = {
    Kind.BOOL: np.uint8, Kind.BYTE: np.uint8, Kind.INT16: np.int16, Kind.INT32: np.int32,
    Kind.INT64: np.int64, Kind.UINT16: np.uint16, Kind.UINT32: np.uint32,
    Kind.UINT64: np.uint64, Kind.FLOAT32: np.uint32, Kind.FLOAT64: np.uint64,
    Kind.BIN64: np.uint8, Kind.BIN128: np.uint8, Kind.BIN256: np.uint8,
    Kind.STRING: np.uint32, Kind.BYTES: np.uint32, Kind.LIST: np.uint32, Kind.ANY: np.uint32,
}

VARLEN = (Kind.STRING, Kind.BYTES)


@dataclass(frozen=True)
class Field:
    tag: int
    kind: Kind
    name: str = ""

    @property
    def width(self) -> int:
        return WIDTH[self.kind]


class Schema:
    def __init__(self, fields):
        fields = [f if isinstance(f, Field) else Field(*f) for f in fields]
        if len(fields) > SPEC_MAX_FIELDS:
            raise ValueError(f"at most {SPEC_MAX_FIELDS} fields")
        self.fields = tuple(Field(f.tag, Kind(f.kind), f.name) for f in fields)
        c = SpecSchema()
        c.nfields = len(self.fields)
        for i, f in enumerate(self.fields):
            c.fields[i].tag = f.tag
            c.fields[i].kind = int(f.kind)
        self.c = c

    def __len__(self):
        return len(self.fields)

    @property
    def tags(self):
        return [f.tag for f in self.fields]

    @property
    def kinds(self):
        return [int(f.kind) for f in self.fields]

    @property
    def widths(self):
        return [f.width for f in self.fields]

    @property
    def column_bytes(self) -> int:
        return sum(self.widths)


# The benchmark schema (SURVEY.md §8(d) "Flat16"): tags 1..16 written in tag order.
FLAT16 = Schema([
    Field(1, Kind.BOOL, "bool"),
    Field(2, Kind.BYTE, "byte"),
    Field(3, Kind.INT16, "int16"),
    Field(4, Kind.INT32, "int32"),
    Field(5, Kind.INT64, "int64"),
    Field(6, Kind.UINT16, "uint16"),
    Field(7, Kind.UINT32, "uint32"),
    Field(8, Kind.UINT64, "uint64"),
    Field(9, Kind.FLOAT32, "float32"),
    Field(10, Kind.FLOAT64, "float64"),
    Field(11, Kind.BIN64, "bin64"),
    Field(12, Kind.BIN128, "bin128"),
    Field(13, Kind.BIN256, "bin256"),
    Field(14, Kind.STRING, "string"),
    Field(15, Kind.BYTES, "bytes"),
    Field(16, Kind.INT64, "int64b"),
])


class NestedSchema:
    """A message with one list<message> field (include/spec_amd.h spec_nested_schema):
    `outer` in write order with exactly one Kind.LIST field, `item` the list items' fields."""

    def __init__(self, outer, item):
        from ._lib import SpecNestedSchema

        self.outer = Schema(outer) if not isinstance(outer, Schema) else outer
        self.item = Schema(item) if not isinstance(item, Schema) else item
        from ._lib import SPEC_NESTED_MAX_FIELDS

        from ._lib import SPEC_TREE_MAX_FIELDS

        if max(len(self.outer), len(self.item)) > SPEC_NESTED_MAX_FIELDS:
            raise ValueError(f"a nested schema's outer and item hold at most {SPEC_NESTED_MAX_FIELDS} fields each")
        # a half of more than 64 fields encodes as one schema tree (check_nested, capi.hip)
        if max(len(self.outer), len(self.item)) > 64 and len(self.outer) + len(self.item) > SPEC_TREE_MAX_FIELDS:
            raise ValueError(f"a nested schema with a half of more than 64 fields holds at most "
                             f"{SPEC_TREE_MAX_FIELDS} fields in all")
        lists = [i for i, f in enumerate(self.outer.fields) if f.kind == Kind.LIST]
        if len(lists) != 1 or any(f.kind == Kind.LIST for f in self.item.fields):
            raise ValueError("outer needs exactly one Kind.LIST field; items must be flat")
        self.list_field = lists[0]
        self.c = SpecNestedSchema()
        self.c.outer = self.outer.c
        self.c.item = self.item.c


# SURVEY.md §8(d) "Nested" (config 4): outer {1 bin128 id, 2 int64 seq, 3 string name,
# 4 list<Item>}, Item {1 int32 key, 2 float64 value, 3 string label}.
NESTED = NestedSchema(
    [Field(1, Kind.BIN128, "id"), Field(2, Kind.INT64, "seq"), Field(3, Kind.STRING, "name"),
     Field(4, Kind.LIST, "items")],
    [Field(1, Kind.INT32, "key"), Field(2, Kind.FLOAT64, "value"), Field(3, Kind.STRING, "label")],
)
