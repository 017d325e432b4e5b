"""ctypes binding of the CPU oracle (oracle/build/libspec_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product path (spec_amd/) never imports this module.

Every helper mirrors one reference function; see the C sources for file:line citations.
Decoders take the bytes of a value that ENDS at len(b) and return (value, n, err) with
err None or the reference's error text.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libspec_oracle.so")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


u8p = C.POINTER(C.c_uint8)


class MessageTable(C.Structure):
    _fields_ = [("table", u8p), ("table_len", C.c_size_t), ("data", C.c_uint32), ("big", C.c_int)]


class ListTable(C.Structure):
    _fields_ = [("table", u8p), ("table_len", C.c_size_t), ("data", C.c_uint32), ("big", C.c_int)]


class MessageField(C.Structure):
    _fields_ = [("tag", C.c_uint16), ("offset", C.c_uint32)]


class ListElement(C.Structure):
    _fields_ = [("offset", C.c_uint32)]


class CMessage(C.Structure):
    _fields_ = [("table", MessageTable), ("bytes", u8p), ("len", C.c_size_t)]


class CList(C.Structure):
    _fields_ = [("table", ListTable), ("bytes", u8p), ("len", C.c_size_t)]


class Buf(C.Structure):
    _fields_ = [("data", u8p), ("len", C.c_size_t), ("cap", C.c_size_t), ("owned", C.c_int),
                ("overflow", C.c_int)]


_SCALARS = {
    "bool": C.c_int, "byte": C.c_uint8, "int16": C.c_int16, "int32": C.c_int32,
    "int64": C.c_int64, "uint16": C.c_uint16, "uint32": C.c_uint32, "uint64": C.c_uint64,
    "float32": C.c_float, "float64": C.c_double,
}


def _declare(L):
    L.so_buf_new.restype = C.POINTER(Buf)
    L.so_buf_new.argtypes = [C.c_size_t]
    L.so_buf_free.argtypes = [C.POINTER(Buf)]
    for name, ct in _SCALARS.items():
        f = getattr(L, f"so_encode_{name}")
        f.restype = C.c_char_p
        f.argtypes = [C.POINTER(Buf), ct, C.POINTER(C.c_int)]
        d = getattr(L, f"so_decode_{name}")
        d.restype = C.c_char_p
        d.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(ct), C.POINTER(C.c_int)]
        g = getattr(L, f"so_message_{name}")
        g.restype = ct
        g.argtypes = [C.POINTER(CMessage), C.c_uint16]
        wf = getattr(L, f"so_field_{name}")
        wf.restype = C.c_char_p
        wf.argtypes = [C.c_void_p, C.c_uint16, ct]
    for w in (64, 128, 256):
        f = getattr(L, f"so_encode_bin{w}")
        f.restype = C.c_char_p
        f.argtypes = [C.POINTER(Buf), C.c_char_p, C.POINTER(C.c_int)]
        d = getattr(L, f"so_decode_bin{w}")
        d.restype = C.c_char_p
        d.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.POINTER(C.c_int)]
        g = getattr(L, f"so_message_bin{w}")
        g.restype = None
        g.argtypes = [C.POINTER(CMessage), C.c_uint16, C.c_char_p]
        wf = getattr(L, f"so_field_bin{w}")
        wf.restype = C.c_char_p
        wf.argtypes = [C.c_void_p, C.c_uint16, C.c_char_p]
    for name in ("bytes", "string"):
        f = getattr(L, f"so_encode_{name}")
        f.restype = C.c_char_p
        f.argtypes = [C.POINTER(Buf), C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
        d = getattr(L, f"so_decode_{name}")
        d.restype = C.c_char_p
        d.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t), C.POINTER(C.c_size_t),
                      C.POINTER(C.c_int)]
        g = getattr(L, f"so_message_{name}")
        g.restype = C.c_void_p
        g.argtypes = [C.POINTER(CMessage), C.c_uint16, C.POINTER(C.c_size_t)]
        wf = getattr(L, f"so_field_{name}")
        wf.restype = C.c_char_p
        wf.argtypes = [C.c_void_p, C.c_uint16, C.c_char_p, C.c_size_t]
    L.so_encode_struct.restype = C.c_char_p
    L.so_encode_struct.argtypes = [C.POINTER(Buf), C.c_int64, C.POINTER(C.c_int)]
    L.so_encode_list_table.restype = C.c_char_p
    L.so_encode_list_table.argtypes = [C.POINTER(Buf), C.c_int64, C.POINTER(ListElement),
                                       C.c_size_t, C.POINTER(C.c_int)]
    L.so_encode_message_table.restype = C.c_char_p
    L.so_encode_message_table.argtypes = [C.POINTER(Buf), C.c_int64, C.POINTER(MessageField),
                                          C.c_size_t, C.POINTER(C.c_int)]
    L.so_decode_type.restype = C.c_char_p
    L.so_decode_type.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_uint8), C.POINTER(C.c_int)]
    L.so_decode_type_size.restype = C.c_char_p
    L.so_decode_type_size.argtypes = L.so_decode_type.argtypes
    L.so_decode_struct.restype = C.c_char_p
    L.so_decode_struct.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.so_decode_list_table.restype = C.c_char_p
    L.so_decode_list_table.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(ListTable), C.POINTER(C.c_int)]
    L.so_decode_message_table.restype = C.c_char_p
    L.so_decode_message_table.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(MessageTable),
                                          C.POINTER(C.c_int)]
    L.so_message_table_len.argtypes = [C.POINTER(MessageTable)]
    L.so_message_table_field.argtypes = [C.POINTER(MessageTable), C.c_int, C.POINTER(MessageField)]
    L.so_message_table_offset.restype = C.c_int64
    L.so_message_table_offset.argtypes = [C.POINTER(MessageTable), C.c_uint16]
    L.so_list_table_len.argtypes = [C.POINTER(ListTable)]
    L.so_list_table_offset.argtypes = [C.POINTER(ListTable), C.c_int, C.POINTER(C.c_int64),
                                       C.POINTER(C.c_int64)]
    L.so_reverse_uint32.restype = C.c_uint32
    L.so_reverse_uint32.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
    L.so_reverse_uint64.restype = C.c_uint64
    L.so_reverse_uint64.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
    L.so_reverse_int64.restype = C.c_int64
    L.so_reverse_int64.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
    L.so_reverse_size.argtypes = [C.c_char_p, C.c_size_t]
    L.so_put_reverse_uint32.argtypes = [C.c_char_p, C.c_uint32]
    L.so_put_reverse_uint64.argtypes = [C.c_char_p, C.c_uint64]
    L.so_put_reverse_int64.argtypes = [C.c_char_p, C.c_int64]
    L.so_open_message_err.restype = C.c_char_p
    L.so_open_message_err.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(CMessage)]
    L.so_parse_message.restype = C.c_char_p
    L.so_parse_message.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(CMessage), C.POINTER(C.c_int)]
    L.so_message_fields.argtypes = [C.POINTER(CMessage)]
    L.so_message_has_field.argtypes = [C.POINTER(CMessage), C.c_uint16]
    L.so_message_list.argtypes = [C.POINTER(CMessage), C.c_uint16, C.POINTER(CList)]
    L.so_message_message.argtypes = [C.POINTER(CMessage), C.c_uint16, C.POINTER(CMessage)]
    L.so_open_list_err.restype = C.c_char_p
    L.so_open_list_err.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(CList)]
    L.so_list_len.argtypes = [C.POINTER(CList)]
    L.so_list_get_bytes.argtypes = [C.POINTER(CList), C.c_int, C.POINTER(C.c_void_p),
                                    C.POINTER(C.c_size_t)]
    L.so_parse_value.restype = C.c_char_p
    L.so_parse_value.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_int)]
    # writer
    L.so_writer_new.restype = C.c_void_p
    L.so_writer_new.argtypes = [C.POINTER(Buf)]
    L.so_writer_free.argtypes = [C.c_void_p]
    L.so_writer_reset.argtypes = [C.c_void_p, C.POINTER(Buf)]
    L.so_writer_err.restype = C.c_char_p
    L.so_writer_err.argtypes = [C.c_void_p]
    for name in ("so_writer_begin_message", "so_writer_begin_list", "so_elem_begin_list",
                 "so_elem_begin_message"):
        getattr(L, name).restype = C.c_char_p
        getattr(L, name).argtypes = [C.c_void_p]
    for name in ("so_field_begin_list", "so_field_begin_message"):
        getattr(L, name).restype = C.c_char_p
        getattr(L, name).argtypes = [C.c_void_p, C.c_uint16]
    L.so_field_any.restype = C.c_char_p
    L.so_field_any.argtypes = [C.c_void_p, C.c_uint16, C.c_char_p, C.c_size_t]
    L.so_writer_has_field.argtypes = [C.c_void_p, C.c_uint16]
    L.so_writer_list_len.argtypes = [C.c_void_p]
    L.so_elem_int64.restype = C.c_char_p
    L.so_elem_int64.argtypes = [C.c_void_p, C.c_int64]
    L.so_elem_string.restype = C.c_char_p
    L.so_elem_string.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    L.so_elem_any.restype = C.c_char_p
    L.so_elem_any.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    L.so_value_int64.restype = C.c_char_p
    L.so_value_int64.argtypes = [C.c_void_p, C.c_int64]
    L.so_value_string.restype = C.c_char_p
    L.so_value_string.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
    L.so_writer_end.restype = C.c_char_p
    L.so_writer_end.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.so_message_stack_new.restype = C.c_void_p
    L.so_message_stack_free.argtypes = [C.c_void_p]
    L.so_message_stack_insert.argtypes = [C.c_void_p, C.c_int, C.c_uint16, C.c_uint32]
    L.so_message_stack_pop.argtypes = [C.c_void_p, C.c_int, C.POINTER(MessageField), C.c_int]
    L.so_message_stack_has_field.argtypes = [C.c_void_p, C.c_int, C.c_uint16]
    L.so_is_big_message.argtypes = [C.POINTER(MessageField), C.c_size_t]
    L.so_is_big_list.argtypes = [C.POINTER(ListElement), C.c_size_t]
    # batch
    L.so_decode_flat_batch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_uint64, C.POINTER(C.c_void_p), C.c_void_p, C.c_int]
    L.so_encode_flat_batch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_void_p),
                                       C.POINTER(C.c_void_p), C.c_uint64, C.c_void_p, C.c_uint64,
                                       C.c_void_p]
    L.so_encode_nested_batch.argtypes = [C.c_void_p] * 9 + [C.c_uint64, C.c_void_p, C.c_uint64,
                                                            C.c_void_p]
    L.so_decode_nested_counts.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    L.so_decode_nested_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64] + [C.c_void_p] * 9
    L.so_encode_flat_batch_mt.argtypes = L.so_encode_flat_batch.argtypes + [C.c_int]
    L.so_encode_nested_batch_mt.argtypes = L.so_encode_nested_batch.argtypes + [C.c_int]
    L.so_decode_nested_batch_mt.argtypes = L.so_decode_nested_batch.argtypes + [C.c_int]
    L.so_parse_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p, C.c_void_p]
    L.so_parse_batch_root.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                      C.c_void_p]
    L.so_decode_flat_errors.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                        C.c_void_p]
    L.so_tree_layout.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.POINTER(C.c_int), C.c_void_p, C.POINTER(C.c_int)]
    L.so_decode_tree_batch.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    L.so_decode_tree_spans.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                                       C.c_void_p]
    L.so_kind_width.argtypes = [C.c_int]
    L.so_decode_values.argtypes = [C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    L.so_encode_tree_batch.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                       C.c_void_p]
    L.so_frames_read.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
    L.so_frames_read.restype = C.c_longlong
    # lz4 (oracle/lz4.c)
    L.so_xxh32.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
    L.so_xxh32.restype = C.c_uint32
    for name in ("so_lz4_decompress_block", "so_lz4_compress_block"):
        getattr(L, name).argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        getattr(L, name).restype = C.c_longlong
    L.so_lz4_frame_write.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_uint32, C.c_int, C.c_int, C.c_int,
                                     C.c_void_p, C.c_size_t]
    L.so_lz4_frame_write.restype = C.c_longlong
    L.so_lz4_frame_read.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t),
                                    C.POINTER(C.c_size_t)]


def _e(err):
    return None if err is None else err.decode()


# ---------------------------------------------------------------- encoders

def _with_buf(fn):
    L = lib()
    b = L.so_buf_new(64)
    try:
        n = C.c_int(0)
        err = fn(L, b, n)
        data = C.string_at(b.contents.data, b.contents.len)
        return data, n.value, _e(err)
    finally:
        L.so_buf_free(b)


def encode(kind: str, v):
    """spec.Encode<Kind>(buf, v) -> (bytes, n, err)"""
    if kind in _SCALARS:
        return _with_buf(lambda L, b, n: getattr(L, f"so_encode_{kind}")(b, v, C.byref(n)))
    if kind.startswith("bin"):
        return _with_buf(lambda L, b, n: getattr(L, f"so_encode_{kind}")(b, bytes(v), C.byref(n)))
    if kind in ("bytes", "string"):
        raw = v.encode() if isinstance(v, str) else bytes(v)
        return _with_buf(lambda L, b, n: getattr(L, f"so_encode_{kind}")(b, raw, len(raw), C.byref(n)))
    if kind == "struct":
        return _with_buf(lambda L, b, n: L.so_encode_struct(b, v, C.byref(n)))
    raise ValueError(kind)


def encode_message_table(data_size: int, fields):
    """EncodeMessageTable(buf, dataSize, fields) -> (trailer bytes, n, err); fields = [(tag, off)]"""
    arr = (MessageField * max(1, len(fields)))(*[MessageField(t, o) for t, o in fields])
    return _with_buf(lambda L, b, n: L.so_encode_message_table(b, data_size, arr, len(fields),
                                                               C.byref(n)))


def encode_list_table(data_size: int, offsets):
    arr = (ListElement * max(1, len(offsets)))(*[ListElement(o) for o in offsets])
    return _with_buf(lambda L, b, n: L.so_encode_list_table(b, data_size, arr, len(offsets), C.byref(n)))


def put_reverse_uint32(v: int) -> bytes:
    p = C.create_string_buffer(5)
    n = lib().so_put_reverse_uint32(p, v)
    return p.raw[5 - n:]


def put_reverse_uint64(v: int) -> bytes:
    p = C.create_string_buffer(10)
    n = lib().so_put_reverse_uint64(p, v)
    return p.raw[10 - n:]


def put_reverse_int64(v: int) -> bytes:
    p = C.create_string_buffer(10)
    n = lib().so_put_reverse_int64(p, v)
    return p.raw[10 - n:]


def reverse_uint32(b: bytes):
    n = C.c_int(0)
    v = lib().so_reverse_uint32(b, len(b), C.byref(n))
    return v, n.value


def reverse_uint64(b: bytes):
    n = C.c_int(0)
    v = lib().so_reverse_uint64(b, len(b), C.byref(n))
    return v, n.value


def reverse_int64(b: bytes):
    n = C.c_int(0)
    v = lib().so_reverse_int64(b, len(b), C.byref(n))
    return v, n.value


def reverse_size(b: bytes) -> int:
    return lib().so_reverse_size(b, len(b))


# ---------------------------------------------------------------- decoders

def decode(kind: str, b: bytes):
    """spec.Decode<Kind>(b) -> (value, n, err)"""
    L = lib()
    n = C.c_int(0)
    if kind in _SCALARS:
        v = _SCALARS[kind]()
        err = getattr(L, f"so_decode_{kind}")(b, len(b), C.byref(v), C.byref(n))
        val = v.value
        if kind == "bool":
            val = bool(val)
        return val, n.value, _e(err)
    if kind.startswith("bin"):
        w = int(kind[3:]) // 8
        out = C.create_string_buffer(w)
        err = getattr(L, f"so_decode_{kind}")(b, len(b), out, C.byref(n))
        return out.raw, n.value, _e(err)
    if kind in ("bytes", "string"):
        off, ln = C.c_size_t(0), C.c_size_t(0)
        err = getattr(L, f"so_decode_{kind}")(b, len(b), C.byref(off), C.byref(ln), C.byref(n))
        raw = b[off.value:off.value + ln.value]
        return (raw.decode("latin-1") if kind == "string" else raw), n.value, _e(err)
    if kind == "struct":
        ds = C.c_int(0)
        err = L.so_decode_struct(b, len(b), C.byref(ds), C.byref(n))
        return ds.value, n.value, _e(err)
    if kind == "type":
        t = C.c_uint8(0)
        err = L.so_decode_type(b, len(b), C.byref(t), C.byref(n))
        return t.value, n.value, _e(err)
    if kind == "type_size":
        t = C.c_uint8(0)
        err = L.so_decode_type_size(b, len(b), C.byref(t), C.byref(n))
        return t.value, n.value, _e(err)
    raise ValueError(kind)


def decode_message_table(b: bytes):
    """DecodeMessageTable(b) -> (fields[(tag,off)], dataSize, big, n, err)"""
    L = lib()
    t = MessageTable()
    n = C.c_int(0)
    buf = C.create_string_buffer(b, len(b))
    err = L.so_decode_message_table(buf, len(b), C.byref(t), C.byref(n))
    fields = []
    for i in range(L.so_message_table_len(C.byref(t))):
        f = MessageField()
        L.so_message_table_field(C.byref(t), i, C.byref(f))
        fields.append((f.tag, f.offset))
    return fields, t.data, bool(t.big), n.value, _e(err)


def decode_list_table(b: bytes):
    """DecodeListTable(b) -> (offsets, dataSize, big, n, err)"""
    L = lib()
    t = ListTable()
    n = C.c_int(0)
    buf = C.create_string_buffer(b, len(b))
    err = L.so_decode_list_table(buf, len(b), C.byref(t), C.byref(n))
    offs = []
    for i in range(L.so_list_table_len(C.byref(t))):
        s, e = C.c_int64(0), C.c_int64(0)
        L.so_list_table_offset(C.byref(t), i, C.byref(s), C.byref(e))
        offs.append(e.value)
    return offs, t.data, bool(t.big), n.value, _e(err)


def parse_value(b: bytes):
    n = C.c_int(0)
    err = lib().so_parse_value(b, len(b), C.byref(n))
    return n.value, _e(err)


class Message:
    """types.Message over a private copy of b (OpenMessageErr semantics)."""

    def __init__(self, b: bytes):
        self._buf = C.create_string_buffer(b, len(b))
        self._base = C.addressof(self._buf)
        self.m = CMessage()
        self.err = _e(lib().so_open_message_err(self._buf, len(b), C.byref(self.m)))

    def fields(self):
        return lib().so_message_fields(C.byref(self.m))

    def has_field(self, tag):
        return bool(lib().so_message_has_field(C.byref(self.m), tag))

    def get(self, kind: str, tag: int):
        L = lib()
        if kind in _SCALARS:
            v = getattr(L, f"so_message_{kind}")(C.byref(self.m), tag)
            return bool(v) if kind == "bool" else v
        if kind.startswith("bin"):
            out = C.create_string_buffer(int(kind[3:]) // 8)
            getattr(L, f"so_message_{kind}")(C.byref(self.m), tag, out)
            return out.raw
        if kind in ("bytes", "string"):
            ln = C.c_size_t(0)
            p = getattr(L, f"so_message_{kind}")(C.byref(self.m), tag, C.byref(ln))
            if not p:
                return None
            return C.string_at(p, ln.value)
        raise ValueError(kind)

    def list_items(self, tag: int):
        """m.List(tag) -> [bytes of each element or None]"""
        L = lib()
        lst = CList()
        L.so_message_list(C.byref(self.m), tag, C.byref(lst))
        out = []
        for i in range(L.so_list_len(C.byref(lst))):
            p, ln = C.c_void_p(), C.c_size_t(0)
            rc = L.so_list_get_bytes(C.byref(lst), i, C.byref(p), C.byref(ln))
            out.append(None if rc < 0 or not p.value else C.string_at(p.value, ln.value))
        return out


class Writer:
    """internal/writer stack machine over a growable buffer."""

    def __init__(self):
        L = lib()
        self.buf = L.so_buf_new(64)
        self.w = L.so_writer_new(self.buf)

    def close(self):
        L = lib()
        if self.w:
            L.so_writer_free(self.w)
            L.so_buf_free(self.buf)
            self.w = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def err(self):
        return _e(lib().so_writer_err(self.w))

    def message(self):
        return _e(lib().so_writer_begin_message(self.w))

    def list(self):
        return _e(lib().so_writer_begin_list(self.w))

    def field(self, tag: int, kind: str, v):
        L = lib()
        if kind in _SCALARS or kind.startswith("bin"):
            return _e(getattr(L, f"so_field_{kind}")(self.w, tag, bytes(v) if kind.startswith("bin") else v))
        if kind in ("bytes", "string"):
            raw = v.encode() if isinstance(v, str) else bytes(v)
            return _e(getattr(L, f"so_field_{kind}")(self.w, tag, raw, len(raw)))
        if kind == "any":
            return _e(L.so_field_any(self.w, tag, bytes(v), len(v)))
        raise ValueError(kind)

    def field_list(self, tag: int):
        return _e(lib().so_field_begin_list(self.w, tag))

    def field_message(self, tag: int):
        return _e(lib().so_field_begin_message(self.w, tag))

    def has_field(self, tag: int) -> bool:
        return bool(lib().so_writer_has_field(self.w, tag))

    def elem_int64(self, v):
        return _e(lib().so_elem_int64(self.w, v))

    def elem_string(self, s):
        raw = s.encode() if isinstance(s, str) else bytes(s)
        return _e(lib().so_elem_string(self.w, raw, len(raw)))

    def elem_any(self, b):
        return _e(lib().so_elem_any(self.w, bytes(b), len(b)))

    def elem_message(self):
        return _e(lib().so_elem_begin_message(self.w))

    def elem_list(self):
        return _e(lib().so_elem_begin_list(self.w))

    def list_len(self):
        return lib().so_writer_list_len(self.w)

    def value_int64(self, v):
        return _e(lib().so_value_int64(self.w, v))

    def value_string(self, s):
        raw = s.encode() if isinstance(s, str) else bytes(s)
        return _e(lib().so_value_string(self.w, raw, len(raw)))

    def end(self):
        """end() -> (bytes, err)"""
        p, ln = C.c_void_p(), C.c_size_t(0)
        err = _e(lib().so_writer_end(self.w, C.byref(p), C.byref(ln)))
        data = C.string_at(p.value, ln.value) if p.value else b""
        return data, err

    def bytes(self):
        return C.string_at(self.buf.contents.data, self.buf.contents.len)


# ---------------------------------------------------------------- batch

def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


def decode_flat_batch(tags, kinds, stream: np.ndarray, ends: np.ndarray, widths, nthreads=1):
    """Per-record OpenMessageErr + getters -> (columns list of uint8 [n, width], status)."""
    n = len(ends)
    cols = [np.zeros((n, w), dtype=np.uint8) for w in widths]
    status = np.zeros(n, dtype=np.uint8)
    tags_a = np.asarray(tags, dtype=np.uint16)
    kinds_a = np.asarray(kinds, dtype=np.uint8)
    colptrs = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    rc = lib().so_decode_flat_batch(len(tags), _ptr(tags_a), _ptr(kinds_a), _ptr(stream),
                                    _ptr(ends), n, colptrs, _ptr(status), nthreads)
    assert rc == 0
    return cols, status


def decode_flat_errors(tags, kinds, stream: np.ndarray, ends: np.ndarray) -> np.ndarray:
    """Per record the *Err getters' error bits (bit f = field f's getter errs) -> uint64 [n]; more
    than 64 fields: uint64 [ceil(nfields / 64), n] (row c: fields 64c..64c+63)."""
    n = len(ends)
    words = max(1, (len(tags) + 63) // 64)
    em = np.zeros((words, max(n, 1)), np.uint64)
    tags_a = np.asarray(tags, dtype=np.uint16)
    kinds_a = np.asarray(kinds, dtype=np.uint8)
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    lib().so_decode_flat_errors(len(tags), _ptr(tags_a), _ptr(kinds_a), _ptr(stream) if stream.size else None,
                                _ptr(ends) if n else None, n, _ptr(em))
    return em[0, :n] if words == 1 else em[:, :n]


def encode_flat_batch(tags, kinds, columns, heaps, n, cap=None):
    """Writer per record -> (stream uint8[total], ends uint64[n])."""
    tags_a = np.asarray(tags, dtype=np.uint16)
    kinds_a = np.asarray(kinds, dtype=np.uint8)
    cols = [np.ascontiguousarray(c) for c in columns]
    colptrs = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    hs = [np.ascontiguousarray(h, dtype=np.uint8) if h is not None else np.zeros(1, np.uint8)
          for h in heaps]
    heapptrs = (C.c_void_p * len(hs))(*[h.ctypes.data for h in hs])
    if cap is None:
        # per record: <= 45 bytes per fixed field (bin256 + type + a 6-byte big-table entry) + string
        # headers; string/bytes payloads from the heaps
        cap = 64 + n * (64 + 48 * len(tags)) + sum(int(h.size) for h in hs) * 2
    out = np.zeros(cap, dtype=np.uint8)
    ends = np.zeros(n, dtype=np.uint64)
    rc = lib().so_encode_flat_batch(len(tags), _ptr(tags_a), _ptr(kinds_a), colptrs, heapptrs, n,
                                    _ptr(out), cap, _ptr(ends))
    if rc != 0:
        raise RuntimeError(f"so_encode_flat_batch rc={rc}")
    total = int(ends[-1]) if n else 0
    return out[:total].copy(), ends


def encode_nested_batch(w: dict, cap=None):
    n = len(w["seq"])
    if cap is None:
        cap = 64 + n * 512 + int(w["name_heap"].size + w["label_heap"].size) * 2
    out = np.zeros(cap, dtype=np.uint8)
    ends = np.zeros(n, dtype=np.uint64)
    args = [w["id"], w["seq"], w["name"], w["name_heap"], w["item_begin"], w["key"], w["value"],
            w["label"], w["label_heap"]]
    args = [np.ascontiguousarray(a) for a in args]
    rc = lib().so_encode_nested_batch(*[_ptr(a) for a in args], n, _ptr(out), cap, _ptr(ends))
    if rc != 0:
        raise RuntimeError(f"so_encode_nested_batch rc={rc}")
    total = int(ends[-1]) if n else 0
    return out[:total].copy(), ends


def encode_flat_batch_mt(tags, kinds, columns, heaps, n, cap, nthreads):
    """The Writer loop on nthreads host threads (CPU baseline): -> (out, ends) where thread t's
    records sit in out[t * (cap // nthreads):] with ends relative to that region."""
    tags_a = np.asarray(tags, dtype=np.uint16)
    kinds_a = np.asarray(kinds, dtype=np.uint8)
    cols = [np.ascontiguousarray(c) for c in columns]
    colptrs = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    hs = [np.ascontiguousarray(h, dtype=np.uint8) if h is not None else np.zeros(1, np.uint8) for h in heaps]
    heapptrs = (C.c_void_p * len(hs))(*[h.ctypes.data for h in hs])
    out = np.zeros(cap, dtype=np.uint8)
    ends = np.zeros(n, dtype=np.uint64)

    def run():
        rc = lib().so_encode_flat_batch_mt(len(tags), _ptr(tags_a), _ptr(kinds_a), colptrs, heapptrs, n, _ptr(out),
                                           cap, _ptr(ends), nthreads)
        if rc != 0:
            raise RuntimeError(f"so_encode_flat_batch_mt rc={rc}")

    return run, out, ends


def nested_batch_mt(w: dict, stream: np.ndarray, ends_in: np.ndarray, cap, nthreads):
    """The nested Writer loop and the nested reader loop (OpenMessageErr + outer getters +
    MessageList Len/Get + item getters) on nthreads host threads (CPU baseline) -> (encode(),
    decode()) callables over preallocated buffers."""
    n = len(w["seq"])
    args = [np.ascontiguousarray(w[k]) for k in ("id", "seq", "name", "name_heap", "item_begin", "key", "value",
                                                 "label", "label_heap")]
    out = np.zeros(cap, dtype=np.uint8)
    ends = np.zeros(n, dtype=np.uint64)
    m = int(w["item_begin"][-1])
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends_in = np.ascontiguousarray(ends_in, dtype=np.uint64)
    d = {"id": np.zeros((n, 16), np.uint8), "seq": np.zeros(n, np.int64), "name": np.zeros((n, 2), np.uint32),
         "key": np.zeros(max(m, 1), np.int32), "value": np.zeros(max(m, 1), np.float64),
         "label": np.zeros((max(m, 1), 2), np.uint32), "item_status": np.zeros(max(m, 1), np.uint8),
         "status": np.zeros(n, np.uint8)}
    L = lib()

    def enc():
        rc = L.so_encode_nested_batch_mt(*[_ptr(a) for a in args], n, _ptr(out), cap, _ptr(ends), nthreads)
        if rc != 0:
            raise RuntimeError(f"so_encode_nested_batch_mt rc={rc}")

    def dec():
        L.so_decode_nested_batch_mt(_ptr(stream), _ptr(ends_in), n, _ptr(args[4]), _ptr(d["id"]), _ptr(d["seq"]),
                                    _ptr(d["name"]), _ptr(d["key"]), _ptr(d["value"]), _ptr(d["label"]),
                                    _ptr(d["item_status"]), _ptr(d["status"]), nthreads)

    return enc, dec, out, ends, d


def decode_nested_batch(stream: np.ndarray, ends: np.ndarray):
    n = len(ends)
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    counts = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.uint8)
    L = lib()
    L.so_decode_nested_counts(_ptr(stream), _ptr(ends), n, _ptr(counts), _ptr(status))
    item_begin = np.zeros(n + 1, dtype=np.uint32)
    np.cumsum(counts, out=item_begin[1:])
    m = int(item_begin[-1])
    out = {
        "id": np.zeros((n, 16), np.uint8), "seq": np.zeros(n, np.int64),
        "name": np.zeros((n, 2), np.uint32), "key": np.zeros(max(m, 1), np.int32),
        "value": np.zeros(max(m, 1), np.float64), "label": np.zeros((max(m, 1), 2), np.uint32),
        "item_status": np.zeros(max(m, 1), np.uint8), "status": status,
        "item_begin": item_begin, "counts": counts,
    }
    L.so_decode_nested_batch(_ptr(stream), _ptr(ends), n, _ptr(item_begin), _ptr(out["id"]),
                             _ptr(out["seq"]), _ptr(out["name"]), _ptr(out["key"]),
                             _ptr(out["value"]), _ptr(out["label"]), _ptr(out["item_status"]),
                             _ptr(status))
    for k in ("key", "value", "label", "item_status"):
        out[k] = out[k][:m]
    return out


PARSE_MESSAGE, PARSE_LIST, PARSE_VALUE = 0, 1, 2


def parse_batch(stream: np.ndarray, ends: np.ndarray, head: int = 0, root: int = PARSE_MESSAGE):
    """ParseMessage (root 0), ParseList (1) or ParseValue (2) per record -> (status uint8[n], sizes
    uint32[n]) (spec_parse_batch semantics)."""
    n = len(ends)
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    st = np.zeros(n, np.uint8)
    sz = np.zeros(n, np.uint32)
    lib().so_parse_batch_root(root, _ptr(stream) if stream.size else None, _ptr(ends) if n else None, n, head,
                              _ptr(st), _ptr(sz))
    return st, sz


# ---------------------------------------------------------------- schema trees (tree.c)

TREE_FIELD = np.dtype([("tag", "<u2"), ("kind", "u1"), ("elem", "u1"), ("parent", "<i2"), ("reserved", "<u2")])
TREE_TABLE = np.dtype([("parent", "<i2"), ("field", "<i2"), ("rel", "u1"), ("shape", "u1"), ("first_column", "<u2"),
                       ("ncolumns", "<u2")])
TREE_COLUMN = np.dtype([("table", "<u2"), ("field", "<i2"), ("role", "u1"), ("kind", "u1"), ("width", "<u2")])


def tree_fields(fields) -> np.ndarray:
    """[(tag, kind, elem, parent), ...] -> the so_tree_field array."""
    a = np.zeros(len(fields), TREE_FIELD)
    for i, (tag, kind, elem, parent) in enumerate(fields):
        a[i] = (tag, kind, elem, parent, 0)
    return a


def tree_layout(fields: np.ndarray):
    """so_tree_layout -> (tables, columns) structured arrays, or None for an invalid tree."""
    t = np.zeros(128, TREE_TABLE)  # so_tree MAX_T
    c = np.zeros(2048, TREE_COLUMN)  # so_tree MAX_C
    nt, nc = C.c_int(0), C.c_int(0)
    rc = lib().so_tree_layout(_ptr(fields), len(fields), _ptr(t), C.byref(nt), _ptr(c), C.byref(nc))
    if rc:
        return None
    return t[: nt.value].copy(), c[: nc.value].copy()


def _entries(tables, col, rows):
    return rows[tables[col["table"]]["parent"]] + 1 if col["role"] == 2 else rows[col["table"]]


def decode_tree_batch(fields: np.ndarray, stream: np.ndarray, ends: np.ndarray):
    """Generated reader over every record -> (rows per table, columns in layout order: uint8
    [entries, width])."""
    tables, cols = tree_layout(fields)
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    n = len(ends)
    rows = np.zeros(len(tables), np.uint64)
    sp = _ptr(stream) if stream.size else None
    lib().so_decode_tree_batch(_ptr(fields), len(fields), sp, _ptr(ends) if n else None, n, None, _ptr(rows))
    rows = [int(r) for r in rows]
    out = [np.zeros((max(_entries(tables, c, rows), 1), int(c["width"])), np.uint8) for c in cols]
    ptrs = (C.c_void_p * len(out))(*[o.ctypes.data for o in out])
    rows2 = np.zeros(len(tables), np.uint64)
    lib().so_decode_tree_batch(_ptr(fields), len(fields), sp, _ptr(ends) if n else None, n, ptrs, _ptr(rows2))
    assert [int(r) for r in rows2] == rows
    return rows, [o[: _entries(tables, c, rows)] for o, c in zip(out, cols)]


def _spans_u32(spans: np.ndarray) -> np.ndarray:
    """(off, len) pairs as uint32 [n, 2]: a span column (uint8 [n, 8]) is viewed, not converted."""
    a = np.ascontiguousarray(spans)
    if a.dtype == np.uint8:
        a = a.view(np.uint32)
    return np.ascontiguousarray(a, dtype=np.uint32).reshape(-1, 2)


def decode_tree_spans(fields: np.ndarray, stream: np.ndarray, spans: np.ndarray):
    """Generated reader over value spans (m.Field(tag).Message() of each) -> (rows, columns)."""
    tables, cols = tree_layout(fields)
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    spans = _spans_u32(spans)
    n = len(spans)
    rows = np.zeros(len(tables), np.uint64)
    sp = _ptr(stream) if stream.size else None
    lib().so_decode_tree_spans(_ptr(fields), len(fields), sp, stream.size, _ptr(spans) if n else None, n, None,
                               _ptr(rows))
    rows = [int(r) for r in rows]
    out = [np.zeros((max(_entries(tables, c, rows), 1), int(c["width"])), np.uint8) for c in cols]
    ptrs = (C.c_void_p * len(out))(*[o.ctypes.data for o in out])
    rows2 = np.zeros(len(tables), np.uint64)
    lib().so_decode_tree_spans(_ptr(fields), len(fields), sp, stream.size, _ptr(spans) if n else None, n, ptrs,
                               _ptr(rows2))
    assert [int(r) for r in rows2] == rows
    return rows, [o[: _entries(tables, c, rows)] for o, c in zip(out, cols)]


def decode_values(kind: int, stream: np.ndarray, spans: np.ndarray):
    """Value.<Kind>Err() over value spans -> (values uint8 [n, width], err uint8 [n])."""
    stream = np.ascontiguousarray(stream, dtype=np.uint8)
    spans = _spans_u32(spans)
    n = len(spans)
    out = np.zeros((max(n, 1), int(lib().so_kind_width(int(kind)))), np.uint8)
    err = np.zeros(max(n, 1), np.uint8)
    rc = lib().so_decode_values(int(kind), _ptr(stream) if stream.size else None, stream.size,
                                _ptr(spans) if n else None, n, _ptr(out), _ptr(err))
    assert rc == 0
    return out[:n], err[:n]


def encode_tree_batch(fields: np.ndarray, columns, heaps, n: int, cap=None):
    """Generated Write() per record -> (stream uint8[total], ends uint64[n]).  columns / heaps in
    layout order (heaps None where unused)."""
    cols = [np.ascontiguousarray(c) if c is not None else np.zeros((1, 1), np.uint8) for c in columns]
    hs = [np.ascontiguousarray(h, dtype=np.uint8) if h is not None else None for h in heaps]
    colptrs = (C.c_void_p * len(cols))(*[c.ctypes.data for c in cols])
    heapptrs = (C.c_void_p * len(hs))(*[h.ctypes.data if h is not None else 0 for h in hs])
    if cap is None:
        cap = 256 + sum(int(c.size) for c in cols) * 4 + sum(int(h.size) for h in hs if h is not None) * 2
    out = np.zeros(cap, np.uint8)
    ends = np.zeros(max(n, 1), np.uint64)
    rc = lib().so_encode_tree_batch(_ptr(fields), len(fields), colptrs, heapptrs, n, _ptr(out), cap, _ptr(ends))
    if rc != 0:
        raise RuntimeError(f"so_encode_tree_batch rc={rc}")
    total = int(ends[n - 1]) if n else 0
    return out[:total].copy(), ends[:n].copy()


def frames_read(buf: np.ndarray, cap: int):
    """mpx connReader.read loop over buf (mpx/conn_reader.go:179-194) -> (ends uint64[k] or None
    when more than cap frames are complete, consumed)."""
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    ends = np.zeros(max(cap, 1), np.uint64)
    used = C.c_uint64(0)
    k = lib().so_frames_read(_ptr(buf) if buf.size else None, buf.size, _ptr(ends), cap, C.byref(used))
    if k < 0:
        return None, int(used.value)
    return ends[:k].copy(), int(used.value)


# ---------------------------------------------------------------- lz4 (mpx compression)

def _u8(b) -> np.ndarray:
    return np.ascontiguousarray(np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b,
                                dtype=np.uint8)


def xxh32(data, seed: int = 0) -> int:
    a = _u8(data)
    return int(lib().so_xxh32(_ptr(a) if a.size else None, a.size, seed))


def lz4_compress_block(data) -> bytes:
    a = _u8(data)
    cap = a.size + a.size // 255 + 64
    out = np.zeros(cap, np.uint8)
    n = lib().so_lz4_compress_block(_ptr(a) if a.size else None, a.size, _ptr(out), cap)
    if n < 0:
        raise RuntimeError("lz4 compress")
    return out[:n].tobytes()


def lz4_decompress_block(data, cap: int):
    """-> bytes, or None on a corrupt block (pierrec decodeBlock's error)."""
    a = _u8(data)
    out = np.zeros(max(cap, 1), np.uint8)
    n = lib().so_lz4_decompress_block(_ptr(a) if a.size else None, a.size, _ptr(out), cap)
    return None if n < 0 else out[:n].tobytes()


def lz4_frame_write(data, flush_ends=None, block_max: int = 256 << 10, content_checksum=True, block_checksum=False,
                    close=True) -> np.ndarray:
    """One LZ4 frame as mpx's writer emits it (flush_ends: the Flush() points, default one at the end)."""
    a = _u8(data)
    fe = np.ascontiguousarray(flush_ends if flush_ends is not None else [a.size], dtype=np.uint64)
    cap = a.size + a.size // 255 + 64 + 12 * (a.size // 1024 + len(fe) + 2)
    out = np.zeros(cap, np.uint8)
    n = lib().so_lz4_frame_write(_ptr(a) if a.size else None, _ptr(fe), fe.size, block_max, int(content_checksum),
                                 int(block_checksum), int(close), _ptr(out), cap)
    if n < 0:
        raise RuntimeError("lz4 frame write")
    return out[:n].copy()


def lz4_frame_read(buf, cap: int):
    """-> (rc, decompressed bytes as np.uint8, consumed)."""
    a = _u8(buf)
    out = np.zeros(max(cap, 1), np.uint8)
    ol, used = C.c_size_t(0), C.c_size_t(0)
    rc = lib().so_lz4_frame_read(_ptr(a) if a.size else None, a.size, _ptr(out), cap, C.byref(ol), C.byref(used))
    return rc, out[:ol.value].copy(), used.value
