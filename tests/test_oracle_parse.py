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
