"""The CPU oracle's Writer against the reference's writer tests.

Ported from internal/writer/{writer,stack,msg,list}_test.go: end() error classes, sticky
errors, pushData with unconsumed data, element/field outside a list/message, the message
side stack sorting shuffled inserts by tag, full message/list writes consumed exactly by
DecodeMessageTable/DecodeListTable, and the tie rule for repeated tags
(internal/writer/stack_msg.go:37-61).
"""
from __future__ import annotations

import ctypes as C
import random
import struct

from oracle import oracle as O

MAX_F32 = struct.unpack("<f", struct.pack("<I", 0x7F7FFFFF))[0]


def write_test_message(w):
    """testWriteMessage (internal/writer/msg_test.go:17-44)"""
    rnd = random.Random(1)
    assert w.field(1, "bool", True) is None
    assert w.field(2, "byte", 2) is None
    assert w.field(10, "int32", 2**31 - 1) is None
    assert w.field(11, "int64", 2**63 - 1) is None
    assert w.field(20, "uint32", 2**32 - 1) is None
    assert w.field(21, "uint64", 2**64 - 1) is None
    assert w.field(30, "float32", MAX_F32) is None
    assert w.field(31, "float64", 1.7976931348623157e308) is None
    assert w.field(40, "bin64", rnd.randbytes(8)) is None
    assert w.field(41, "bin128", rnd.randbytes(16)) is None
    assert w.field(42, "bin256", rnd.randbytes(32)) is None
    assert w.field(50, "string", "hello world") is None
    assert w.field(51, "bytes", b"hello world") is None
    assert w.field_list(60) is None
    assert w.elem_string("sublist") is None
    assert w.end()[1] is None
    assert w.field_message(61) is None
    assert w.field(1, "string", "submessage") is None
    assert w.end()[1] is None


def test_message_writer_writes_message():
    w = O.Writer()
    w.message()
    write_test_message(w)
    b, err = w.end()
    assert err is None
    _, _, _, n, err = O.decode_message_table(b)
    assert err is None and n == len(b)
    m = O.Message(b)
    assert m.err is None
    assert m.get("bool", 1) is True and m.get("byte", 2) == 2
    assert m.get("int32", 10) == 2**31 - 1 and m.get("int64", 11) == 2**63 - 1
    assert m.get("uint32", 20) == 2**32 - 1 and m.get("uint64", 21) == 2**64 - 1
    assert m.get("float32", 30) == MAX_F32
    assert m.get("string", 50) == b"hello world" and m.get("bytes", 51) == b"hello world"
    items = m.list_items(60)
    assert len(items) == 1 and O.decode("string", items[0])[0] == "sublist"
    # n == len(b) for a recursive parse too (ParseMessage, internal/types/msg.go:58-82)
    assert O.parse_value(b) == (len(b), None)


def test_list_writer_writes_list():
    """TestListWriter__should_write_list (internal/writer/list_test.go:15-62), int/string subset"""
    w = O.Writer()
    w.list()
    assert w.elem_int64(2**63 - 1) is None
    assert w.elem_string("hello world") is None
    assert w.elem_list() is None
    assert w.elem_string("sublist") is None
    assert w.end()[1] is None
    assert w.elem_message() is None
    assert w.field(1, "string", "submessage") is None
    assert w.end()[1] is None
    b, err = w.end()
    assert err is None
    offs, _, _, n, err = O.decode_list_table(b)
    assert err is None and n == len(b) and len(offs) == 4


def test_copy_reproduces_raw_bytes():
    """TestMessageWriter_Copy (msg_test.go:68-99): re-writing every field of an opened message
    in table order (Copy -> fieldAny) yields identical bytes."""
    w = O.Writer()
    w.message()
    write_test_message(w)
    b, _ = w.end()
    m = O.Message(b)
    w2 = O.Writer()
    w2.message()
    fields, _, _, _, _ = O.decode_message_table(b)
    for tag, end in fields:
        start = 0 if tag == fields[0][0] else [e for t, e in fields if t < tag][-1]
        assert w2.field(tag, "any", b[start:end]) is None
    b2, err = w2.end()
    assert err is None and b2 == b
    assert m.err is None


def test_end_stack_is_empty():
    w = O.Writer()
    _, err = w.end()
    assert err is not None and "stack is empty" in err


def test_end_not_root_value():
    w = O.Writer()
    w.message()
    w.value_int64(1)
    _, err = w.end()
    assert err is not None and "not root value" in err


def test_end_returns_message_bytes():
    w = O.Writer()
    w.message()
    b, err = w.end()
    assert err is None and b[-1] == 80


def test_errors_are_sticky():
    w = O.Writer()
    _, err = w.end()
    assert err is not None
    assert w.message() is not None or w.err() is not None
    assert w.err() is not None


def test_push_data_unconsumed():
    """TestWriter_pushData__should_return_error_when_unconsumed_data (writer_test.go:146-153)"""
    w = O.Writer()
    w.message()
    assert w.value_int64(1) is None
    assert w.value_int64(1) is not None


def test_element_outside_list():
    w = O.Writer()
    assert w.elem_int64(1) is not None
    w = O.Writer()
    w.message()
    assert w.elem_int64(1) is not None


def test_field_outside_message():
    w = O.Writer()
    assert w.field(1, "int64", 1) is not None
    w = O.Writer()
    w.list()
    assert w.field(1, "int64", 1) is not None


def _stack():
    L = O.lib()
    L.so_message_stack_new.restype = C.c_void_p
    L.so_message_stack_free.argtypes = [C.c_void_p]
    L.so_message_stack_insert.argtypes = [C.c_void_p, C.c_int, C.c_uint16, C.c_uint32]
    L.so_message_stack_pop.argtypes = [C.c_void_p, C.c_int, C.POINTER(O.MessageField), C.c_int]
    L.so_message_stack_has_field.argtypes = [C.c_void_p, C.c_int, C.c_uint16]
    return L


def test_message_stack_sorts_shuffled_inserts():
    """TestMessageBuffer_Insert__should_insert_field_into_table_ordered_by_tags
    (internal/writer/stack_test.go:65-112): nested tables on one side stack."""
    L = _stack()
    s = L.so_message_stack_new()
    rnd = random.Random(5)
    matrix = [1, 10, 100, 10, 1, 0, 3]
    offsets, total = [], 0
    for cnt in matrix:
        offsets.append(total)
        ff = [(i + 1, i * 10) for i in range(cnt)]
        rnd.shuffle(ff)
        for tag, off in ff:
            L.so_message_stack_insert(s, total, tag, off)
        total += cnt
    for i in range(len(matrix) - 1, -1, -1):
        out = (O.MessageField * 128)()
        k = L.so_message_stack_pop(s, offsets[i], out, 128)
        assert [(out[j].tag, out[j].offset) for j in range(k)] == [(j + 1, j * 10) for j in range(matrix[i])]
    L.so_message_stack_free(s)


def test_repeated_tag_later_write_sorts_first():
    """stack_msg.go:47-60: an equal tag inserted later moves before the earlier entry."""
    w = O.Writer()
    w.message()
    w.field(5, "int64", 1)
    w.field(5, "int64", 2)
    b, err = w.end()
    assert err is None
    fields, _, _, _, _ = O.decode_message_table(b)
    # data: [int64 1 | int64 2]; the later write (end offset 4) sits first in the table
    assert fields == [(5, 4), (5, 2)]


def test_big_message_when_tag_over_255():
    w = O.Writer()
    w.message()
    w.field(256, "int64", 1)
    b, err = w.end()
    assert err is None and b[-1] == 81
    fields, _, big, _, _ = O.decode_message_table(b)
    assert big and fields == [(256, 2)]
