"""Schema descriptors from .spec text (spec_amd.specfile): field order, kinds, enums as int32,
list<message> as a NestedSchema, unsupported kinds (CPU)."""
from __future__ import annotations

import pytest

from spec_amd import Kind, NestedSchema, Schema
from spec_amd.specfile import load

SPEC = """
import ( "other" )
options ( go_package="example.com/x" )

enum Color {
    NONE = 0;
    RED = 1; // comment
}

// a record
message Record {
    id      bin128  1;
    seq     int64   2;
    name    string  3;
    color   Color   4;
    items   []Item  5;
}

message Item {
    key     int32   1;
    value   float64 2;
    label   string  3;
}

message Flat {
    a bool 1; b byte 2; c uint64 9; d bytes 10; e float32 11;
}

struct Pair { k int32; v int32; }

message WithStruct {
    p Pair 1;
    x int64 2;
}

service Svc {
    method(req Record) (resp Item);
}
"""


def test_flat_and_enum():
    f = load(SPEC)
    s = f.schema("Flat")
    assert isinstance(s, Schema)
    assert [(x.tag, x.kind) for x in s.fields] == [(1, Kind.BOOL), (2, Kind.BYTE), (9, Kind.UINT64),
                                                   (10, Kind.BYTES), (11, Kind.FLOAT32)]
    assert f.enums["Color"] == {"NONE": 0, "RED": 1}


def test_nested_record():
    s = load(SPEC).schema("Record")
    assert isinstance(s, NestedSchema)
    assert [(x.tag, x.kind) for x in s.outer.fields] == [(1, Kind.BIN128), (2, Kind.INT64), (3, Kind.STRING),
                                                         (4, Kind.INT32), (5, Kind.LIST)]
    assert [(x.tag, x.kind) for x in s.item.fields] == [(1, Kind.INT32), (2, Kind.FLOAT64), (3, Kind.STRING)]


def test_unsupported_kinds():
    f = load(SPEC)
    with pytest.raises(ValueError):
        f.schema("WithStruct")
    s = f.schema("WithStruct", skip_unsupported=True)
    assert [(x.tag, x.kind) for x in s.fields] == [(2, Kind.INT64)]
