"""The oracle's batch ParseMessage (spec_parse_messages semantics) against the reference's
ParseValue rules, on hand-built values (CPU)."""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from tests.gpu_helpers import concat_records


def _msg(fields):
    w = O.Writer()
    w.message()
    for tag, kind, v in fields:
        assert w.field(tag, kind, v) is None
    b, err = w.end()
    assert err is None
    return b


def _raw_message(values):
    """A message whose field i is the raw value bytes values[i] (tags 1..n)."""
    data = b"".join(values)
    ends = list(np.cumsum([len(v) for v in values]))
    trailer, _, err = O.encode_message_table(len(data), [(i + 1, int(e)) for i, e in enumerate(ends)])
    assert err is None
    return data + trailer


def test_parse_batch_classes():
    good = _msg([(1, "int64", 5), (2, "string", "abc")])
    inf32 = O.encode("float32", float("inf"))[0]
    bad_int16 = O.put_reverse_int64(40000)[-3:] + bytes([10])  # int16 type, value out of range
    lst_items = O.encode("int64", 1)[0] + O.encode("int64", 2)[0]
    swapped = lst_items + O.encode_list_table(len(lst_items), [4, 2])[0]  # ends decrease: Go panics
    recs = [
        good,                                   # ok
        b"",                                    # empty: ok, size 0
        bytes([0xFF, 80]),                      # invalid table size
        _raw_message([inf32]),                  # float32 +Inf: overflow => nested error
        _raw_message([bad_int16]),              # int16 overflow => nested error
        _raw_message([bytes([1, 2, 3, 99])]),   # unsupported type 99
        _raw_message([swapped]),                # list with start > end => panic
        _raw_message([good]),                   # nested message: ok
    ]
    stream, ends = concat_records(recs)
    st, sz = O.parse_batch(stream, ends)
    assert list(st) == [0, 0, 2, 7, 7, 7, 6, 0]
    assert sz[0] == len(good) and sz[1] == 0 and sz[7] == len(recs[7])


def _list(values):
    """A list whose element i is the raw value bytes values[i] (ListWriter's layout)."""
    data = b"".join(values)
    ends = [int(e) for e in np.cumsum([len(v) for v in values])]
    trailer, _, err = O.encode_list_table(len(data), ends)
    assert err is None
    return data + trailer


def _struct(data: bytes, ds=None):
    """EncodeStruct's layout: data | rvarint(dataSize) | TypeStruct (90); ds < 128."""
    ds = len(data) if ds is None else ds
    return data + bytes([ds, 90])


def parse_cases():
    """Records for ParseList / ParseValue (and their expected status per root)."""
    i64 = O.encode("int64", 7)[0]
    s = O.encode("string", "hey")[0]
    good = _msg([(1, "int64", 5), (2, "string", "abc")])
    lst = _list([i64, s, good, b"", _list([i64])])
    inf32 = O.encode("float32", float("inf"))[0]
    bad_int16 = O.put_reverse_int64(40000)[-3:] + bytes([10])
    swapped = i64 + i64 + O.encode_list_table(2 * len(i64), [len(i64) * 2, len(i64)])[0]
    return {
        "list_ok": lst,
        "list_empty": b"",
        "list_bad_table": bytes([0xFF, 70]),
        "list_nested_bad": _list([i64, inf32]),
        "list_unsupported": _list([bytes([1, 2, 99])]),
        "list_swapped": swapped,
        "list_struct_ok": _list([_struct(b"\x01\x02")]),
        "list_struct_past_slice": _list([_struct(b"\x01", ds=5)]),
        "value_int": i64,
        "value_string": s,
        "value_message": good,
        "value_list": lst,
        "value_empty": b"",
        "value_bad_int16": bad_int16,
        "value_inf32": inf32,
        "value_unsupported": bytes([3, 99]),
        "value_struct_ok": _struct(b"\x05\x06\x07"),
        "value_struct_past_slice": _struct(b"", ds=9),
        "value_message_nested_panic": _raw_message([swapped]),
        "value_bad_message": bytes([0xFF, 80]),
    }


def test_parse_list_and_value_roots():
    """ParseList / ParseValue (internal/types/list.go:35-53, value.go:49-113) per record: the
    root's own error class for a list table (1-5), 7 for any value error, 6 where Go panics
    (a list element whose start > end; value.go:110's b[len(b)-n:] on a struct whose data size
    runs past its slice), sizes = ParseValue's n / the list's bytes."""
    c = parse_cases()
    names = list(c)
    stream, ends = concat_records([c[k] for k in names])
    st_l, sz_l = O.parse_batch(stream, ends, root=O.PARSE_LIST)
    st_v, sz_v = O.parse_batch(stream, ends, root=O.PARSE_VALUE)
    L = dict(zip(names, zip(st_l, sz_l)))
    V = dict(zip(names, zip(st_v, sz_v)))
    assert L["list_ok"] == (0, len(c["list_ok"]))
    assert L["list_empty"] == (0, 0)
    assert L["list_bad_table"][0] == 2  # invalid table size
    assert L["list_nested_bad"][0] == 7 and L["list_unsupported"][0] == 7
    assert L["list_swapped"][0] == 6
    assert L["list_struct_ok"][0] == 0 and L["list_struct_past_slice"][0] == 6
    assert V["value_int"] == (0, len(c["value_int"])) and V["value_string"] == (0, len(c["value_string"]))
    assert V["value_message"] == (0, len(c["value_message"])) and V["value_list"] == (0, len(c["value_list"]))
    assert V["value_empty"][0] == 7 and V["value_unsupported"][0] == 7
    assert V["value_bad_int16"][0] == 7 and V["value_inf32"][0] == 7 and V["value_bad_message"][0] == 7
    assert V["value_struct_ok"] == (0, len(c["value_struct_ok"]))
    assert V["value_struct_past_slice"][0] == 6 and V["value_message_nested_panic"][0] == 6
    # the same bytes as messages: ParseMessage keeps its classes, a struct past its slice panics
    st_m, _ = O.parse_batch(stream, ends)
    assert st_m[names.index("value_message")] == 0
    assert st_m[names.index("value_message_nested_panic")] == 6
