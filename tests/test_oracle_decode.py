"""The CPU oracle against every assertion of the reference's decode tests.

Ported from internal/decode/*_test.go (basecomplextech/spec): round trips at the extremes,
DecodeTypeSize == encoded length, table round trips over format.TestFields/TestElements
suffixes, and the hand-crafted error classes.  Known-answer byte vectors for the worked
examples of SURVEY.md Appendix A are checked too (varint layout: oracle/compactint.c,
"parity unpinned" at the varint byte level — the reference ships no byte vectors).
"""
from __future__ import annotations

import math
import struct

import pytest

import numpy as np
from oracle import oracle as O

T = dict(undefined=0, true=1, false=2, byte=3, int16=10, int32=11, int64=12, uint16=20, uint32=21,
         uint64=22, bin64=30, bin128=31, bin256=32, float32=40, float64=41, bytes=50, string=60,
         list=70, big_list=71, message=80, big_message=81, struct=90)

MAX_F32 = struct.unpack("<f", struct.pack("<I", 0x7F7FFFFF))[0]


def test_fields(big=False, n=10):
    """format.TestFieldsSizeN (internal/format/test_msg.go:23-40)"""
    tag0, off0 = (256, 65536) if big else (0, 0)
    return [(tag0 + i + 1, off0 + i * 10) for i in range(n)]


def test_elements(big=False, n=10):
    """format.TestElementsSizeN (internal/format/test_list.go:23-37)"""
    off0 = 65536 if big else 0
    return [off0 + i * 10 for i in range(n)]


test_fields.__test__ = False
test_elements.__test__ = False


def append_size(b: bytes, size: int) -> bytes:
    """appendSize (internal/decode/type_test.go:43-49)"""
    return b + O.put_reverse_uint32(size)


def roundtrip(kind, v, typ):
    p, n, err = O.encode(kind, v)
    assert err is None and n == len(p)
    got, m, err = O.decode(kind, p)
    assert err is None
    assert m == len(p)
    t, size, err = O.decode("type_size", p)
    assert err is None and t == typ and size == len(p)
    return got


# ---- byte_test.go:18-65
def test_decode_bool():
    for b, want, t in ((bytes([T["true"]]), True, T["true"]), (bytes([T["false"]]), False, T["false"])):
        v, n, err = O.decode("bool", b)
        assert err is None and n == 1 and v is want
        typ, size, err = O.decode("type_size", b)
        assert err is None and typ == t and size == 1


def test_decode_bool_other_type_is_false_without_error():
    # byte.go:38-51: true iff type == TypeTrue, anything else false, no error (Appendix B.1)
    v, n, err = O.decode("bool", bytes([7, T["byte"]]))
    assert v is False and err is None


def test_decode_byte():
    assert roundtrip("byte", 1, T["byte"]) == 1


# ---- int_test.go:18-95
@pytest.mark.parametrize("kind,v", [("int16", 32767), ("int32", 2**31 - 1), ("int64", 2**63 - 1),
                                    ("int16", -32768), ("int32", -2**31), ("int64", -2**63)])
def test_decode_int_extremes(kind, v):
    assert roundtrip(kind, v, T[kind]) == v


def test_decode_int64_from_int32():
    p, _, _ = O.encode("int32", 2**31 - 1)
    v, n, err = O.decode("int64", p)
    assert err is None and n == len(p) and v == 2**31 - 1


def test_decode_int_narrowing_overflow():
    p, _, _ = O.encode("int64", 2**40)
    _, _, err = O.decode("int32", p)
    assert err is not None and "overflow" in err
    p, _, _ = O.encode("int32", 40000)
    _, _, err = O.decode("int16", p)
    assert err is not None and "overflow" in err


# ---- uint_test.go:19-94
@pytest.mark.parametrize("kind,v", [("uint16", 65535), ("uint32", 2**32 - 1), ("uint64", 2**64 - 1),
                                    ("uint16", 0), ("uint64", 0)])
def test_decode_uint_extremes(kind, v):
    assert roundtrip(kind, v, T[kind]) == v


def test_decode_uint64_from_uint32():
    p, _, _ = O.encode("uint32", 2**32 - 1)
    v, n, err = O.decode("uint64", p)
    assert err is None and n == len(p) and v == 2**32 - 1


# ---- float_test.go:19-86
def test_decode_float32():
    assert roundtrip("float32", MAX_F32, T["float32"]) == MAX_F32


def test_decode_float32_from_float64():
    p, _, _ = O.encode("float64", MAX_F32)
    v, n, err = O.decode("float32", p)
    assert err is None and n == len(p) and v == MAX_F32


def test_decode_float64():
    assert roundtrip("float64", 1.7976931348623157e308, T["float64"]) == 1.7976931348623157e308


def test_decode_float64_from_float32():
    p, _, _ = O.encode("float32", MAX_F32)
    v, n, err = O.decode("float64", p)
    assert err is None and n == len(p) and v == MAX_F32


def test_decode_float32_out_of_range_is_error():
    # float.go:15-32: |v| > MaxFloat32 => error (Appendix B.2)
    p, _, _ = O.encode("float64", 1e300)
    _, _, err = O.decode("float32", p)
    assert err is not None
    p, _, _ = O.encode("float32", math.inf)
    _, _, err = O.decode("float32", p)
    assert err is not None


# ---- bin_test.go:19-80
@pytest.mark.parametrize("kind", ["bin64", "bin128", "bin256"])
def test_decode_bin(kind):
    import os

    v = os.urandom(int(kind[3:]) // 8)
    assert roundtrip(kind, v, T[kind]) == v


# ---- string_test.go:18-41, bytes_test.go:18-41
def test_decode_string():
    assert roundtrip("string", "hello, world", T["string"]) == "hello, world"


def test_decode_bytes():
    assert roundtrip("bytes", b"hello, world", T["bytes"]) == b"hello, world"


# ---- type_test.go:18-41
def test_decode_type():
    v, n, err = O.decode("type", bytes([T["string"]]))
    assert err is None and n == 1 and v == T["string"]


def test_decode_type_empty_is_undefined():
    v, n, err = O.decode("type", b"")
    assert err is None and n == 0 and v == T["undefined"]


@pytest.mark.parametrize("kind", ["bool", "byte", "int32", "int64", "uint64", "float64", "string", "bytes"])
def test_decode_empty_input_is_zero(kind):
    # Appendix B.9: len(b)==0 => zero value, n = 0, nil error
    v, n, err = O.decode(kind, b"")
    assert err is None and n == 0 and not v


# ---- msg_test.go:30-143
def test_decode_message_meta():
    fields = test_fields()
    b, _, err = O.encode_message_table(100, fields)
    assert err is None
    b = bytes(100) + b  # buf.Grow(dataSize) before the table
    got, dsize, big, n, err = O.decode_message_table(b)
    assert err is None and n == len(b) and dsize == 100 and len(got) == len(fields)
    typ, size, err = O.decode("type_size", b)
    assert err is None and typ == T["message"] and size == len(b)


@pytest.mark.parametrize("big", [False, True])
def test_decode_message_table_suffixes(big):
    fields = test_fields(big)
    for i in range(len(fields) + 1):
        b, _, err = O.encode_message_table(0, fields[i:])
        assert err is None
        got, _, isbig, _, err = O.decode_message_table(b)
        assert err is None
        assert got == fields[i:]
        assert isbig == (big and i < len(fields))


def test_decode_message_invalid_type():
    b, _, _ = O.encode_message_table(100, test_fields())
    b = bytes(100) + b[:-1] + bytes([T["list"]])
    err = O.decode_message_table(b)[-1]
    assert err is not None and "invalid type" in err


def test_decode_message_invalid_table_size():
    err = O.decode_message_table(bytes([0xFF, T["message"]]))[-1]
    assert err is not None and "invalid table size" in err


def test_decode_message_invalid_data_size():
    b = append_size(bytes([0xFF]), 1000) + bytes([T["message"]])
    err = O.decode_message_table(b)[-1]
    assert err is not None and "invalid data size" in err


def test_decode_message_invalid_table():
    b, _, _ = O.encode_message_table(0, [])
    b = append_size(append_size(b, 0), 1000) + bytes([T["message"]])
    err = O.decode_message_table(b)[-1]
    assert err is not None and "invalid table" in err


def test_decode_message_invalid_data():
    b, _, _ = O.encode_message_table(0, [])
    b = append_size(append_size(b, 1000), 0) + bytes([T["message"]])
    err = O.decode_message_table(b)[-1]
    assert err is not None and "invalid data" in err


# ---- list_test.go:30-143
def test_decode_list_meta():
    elems = test_elements()
    b, _, err = O.encode_list_table(100, elems)
    assert err is None
    b = bytes(100) + b
    offs, dsize, big, n, err = O.decode_list_table(b)
    assert err is None and n == len(b) and dsize == 100 and len(offs) == len(elems)
    typ, size, err = O.decode("type_size", b)
    assert err is None and typ == T["list"] and size == len(b)


@pytest.mark.parametrize("big", [False, True])
def test_decode_list_table_suffixes(big):
    elems = test_elements(big)
    for i in range(len(elems) + 1):
        b, _, err = O.encode_list_table(0, elems[i:])
        assert err is None
        offs, _, _, _, err = O.decode_list_table(b)
        assert err is None and offs == elems[i:]


def test_is_big_list_counts_elements():
    # Appendix B.7: a 256-element list of tiny items is big (list.go:40-54)
    b, _, _ = O.encode_list_table(0, list(range(1, 256)))
    assert O.decode_list_table(b)[2] is False
    b, _, _ = O.encode_list_table(0, list(range(1, 257)))
    assert O.decode_list_table(b)[2] is True


@pytest.mark.parametrize("name,b", [
    ("invalid table size", bytes([0xFF, T["list"]])),
    ("invalid data size", append_size(bytes([0xFF]), 1000) + bytes([T["list"]])),
    ("invalid table", append_size(append_size(b"", 0), 1000) + bytes([T["list"]])),
    ("invalid data", append_size(append_size(b"", 1000), 0) + bytes([T["list"]])),
])
def test_decode_list_errors(name, b):
    err = O.decode_list_table(b)[-1]
    assert err is not None and name in err


def test_decode_list_invalid_type():
    b, _, _ = O.encode_list_table(100, test_elements())
    b = bytes(100) + b[:-1] + bytes([T["message"]])
    err = O.decode_list_table(b)[-1]
    assert err is not None and "invalid type" in err


# ---- known-answer vectors (under the compactint reconstruction)
def test_kat_string_hello_world():
    b, n, err = O.encode("string", "hello, world")
    assert b.hex() == "68656c6c6f2c20776f726c64000c3c" and n == 15


def test_kat_message_bool_int32():
    w = O.Writer()
    assert w.message() is None
    assert w.field(1, "bool", True) is None
    assert w.field(2, "int32", -1) is None
    data, err = w.end()
    assert err is None
    assert data.hex() == "01010b010001020003030650"


@pytest.mark.parametrize("v,hexs", [(0, "00"), (1, "01"), (127, "7f"), (128, "0180"), (300, "02ac"),
                                    (2**32 - 1, "0fffffffff")])
def test_kat_reverse_uint32(v, hexs):
    b = O.put_reverse_uint32(v)
    assert b.hex() == hexs
    got, n = O.reverse_uint32(b)
    assert got == v and n == len(b)


def test_reverse_varint_incomplete_is_negative():
    # a lone 0xff: "invalid table size" needs n < 0 (internal/decode/msg_test.go:88-97)
    _, n = O.reverse_uint32(bytes([0xFF]))
    assert n < 0
    _, n = O.reverse_uint64(bytes([0xFF] * 11))
    assert n < 0


def test_signed_zigzag():
    for v in (0, -1, 1, -64, 63, -2**63, 2**63 - 1):
        b = O.put_reverse_int64(v)
        got, n = O.reverse_int64(b)
        assert got == v and n == len(b)


def test_err_getters_mask():
    """*Err getters (internal/types/msg.go:233-459): an absent field is no error (field(tag) is
    nil => Decode on empty input), a type mismatch is; bool never errs (byte.go:38-51)."""
    w = O.Writer()
    w.message()
    assert w.field(1, "int64", 1 << 40) is None   # read as int32: overflow
    assert w.field(2, "string", "x") is None      # read as int64: invalid type
    assert w.field(3, "bool", True) is None       # read as bool: fine
    assert w.field(4, "uint16", 7) is None        # read as uint64: cross-width fine
    data, err = w.end()
    w.close()
    stream = np.frombuffer(data, np.uint8)
    ends = np.array([len(data)], np.uint64)
    mask = O.decode_flat_errors([1, 2, 3, 4, 5], [4, 5, 1, 8, 4], stream, ends)  # tag 5 absent
    assert int(mask[0]) == 0b00011
