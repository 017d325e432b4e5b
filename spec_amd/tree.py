"""Schema trees: batch decode/encode of messages with every kind a generated reader/writer
handles — structs, enums, sub-messages, value lists, lists of structs and of messages, any
(host side of include/spec_amd.h spec_tree_*).

A schema is described with the .spec language's shapes (internal/lang/parser/grammar.y):

    Struct("Struct", [("key", Kind.INT32), ("value", Kind.INT32)])
    Message("Submessage", [("value", 1, Kind.STRING), ("next", 2, <Message>)])
    ListOf(Kind.INT64), ListOf(<Struct>), ListOf(<Message>), Kind.ANY

and flattened into the tree the C ABI takes (`Tree`).  A recursive message (pkg1.spec's
Submessage.next) is unrolled `max_depth` times: beyond that the field is not read (a reader
only opens what it accesses) and not written.

Decoded output is a set of tables (spec_tree_layout): the records, one table per sub-message
field (a row per owner row) and one per list field (a row per element, CSR `#begin`).  Column
names: `a.b` (a field), `a.b.m` (struct member), `l[]` (value list elements), `l[].x` (item
field / struct member), `a?` (HasField of a message or list field), `l#begin`, `<table>#status`
(`#status` for the records), `<table>#errmask` (per message row: bit k = the k-th direct
field's *Err getter errs), `a#type` (Value.Type() of an `any` field).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from .schema import WIDTH, Kind

SCALARS = tuple(Kind(k) for k in range(1, 16))
REL_ROOT, REL_ONE, REL_MANY = 0, 1, 2
SHAPE_MESSAGE, SHAPE_VALUE, SHAPE_STRUCT = 0, 1, 2
ROLE_VALUE, ROLE_PRESENT, ROLE_BEGIN, ROLE_STATUS, ROLE_ERRMASK, ROLE_TYPE = 0, 1, 2, 3, 4, 5
INPUT_ROLES = (ROLE_VALUE, ROLE_PRESENT, ROLE_BEGIN)  # what spec_encode_tree reads


class Struct:
    """A .spec struct: members in declaration order, each a scalar kind (Kind.INT32 for an enum)
    or another Struct ("structs support only value types or other structs",
    internal/lang/model/struct_field.go:57-70)."""

    def __init__(self, name: str, members):
        self.name = name
        self.members = [(m, k if isinstance(k, Struct) else Kind(k)) for m, k in members]
        for _, k in self.members:
            if not isinstance(k, Struct) and k not in SCALARS:
                raise ValueError(f"struct {name}: members must be scalar kinds or structs")


class Message:
    """A .spec message: (name, tag, type) in write order; type = a Kind (Kind.INT32 for an enum,
    Kind.ANY for `any`), a Struct, a Message or a ListOf.  `fields` may be set after creation
    (recursive messages)."""

    def __init__(self, name: str, fields=None):
        self.name = name
        self.fields = list(fields or [])


@dataclass(frozen=True)
class ListOf:
    elem: object  # Kind (scalar), Struct or Message


@dataclass
class TreeField:
    path: str
    tag: int
    kind: Kind
    elem: int = 0
    parent: int = -1


@dataclass
class TreeTable:
    index: int
    path: str
    parent: int
    field: int
    rel: int
    shape: int
    columns: list = field(default_factory=list)


@dataclass
class TreeColumn:
    index: int
    name: str
    table: int
    field: int
    role: int
    kind: int
    width: int


class Tree:
    """A record message flattened into spec_tree fields (pre-order), with its table/column layout
    from spec_tree_layout."""

    def __init__(self, root: Message, max_depth: int = 2):
        self.root = root
        self.fields: list[TreeField] = []
        self._add_message(root, -1, "", {root.name: 1}, max_depth)
        if len(self.fields) > _lib.SPEC_TREE_MAX_FIELDS:
            raise ValueError("tree too large")
        c = _lib.SpecTree()
        c.nfields = len(self.fields)
        for i, f in enumerate(self.fields):
            c.fields[i].tag = f.tag
            c.fields[i].kind = int(f.kind)
            c.fields[i].elem = int(f.elem)
            c.fields[i].parent = f.parent
        self.c = c
        self._layout()

    @classmethod
    def from_fields(cls, fields):
        """A tree from flattened fields [(path, tag, kind, elem, parent), ...] (pre-order)."""
        t = cls.__new__(cls)
        t.root = None
        t.fields = [TreeField(p, tag, Kind(k), int(e), par) for p, tag, k, e, par in fields]
        c = _lib.SpecTree()
        c.nfields = len(t.fields)
        for i, f in enumerate(t.fields):
            c.fields[i].tag, c.fields[i].kind, c.fields[i].elem, c.fields[i].parent = f.tag, int(f.kind), f.elem, f.parent
        t.c = c
        t._layout()
        return t

    def to_fields(self):
        return [(f.path, f.tag, int(f.kind), int(f.elem), f.parent) for f in self.fields]

    # -- flattening --
    def _add(self, path, tag, kind, elem=0, parent=-1):
        self.fields.append(TreeField(path, tag, Kind(kind), int(elem), parent))
        return len(self.fields) - 1

    def _add_message(self, msg, parent, prefix, depth, max_depth):
        for name, tag, typ in msg.fields:
            path = prefix + name
            if isinstance(typ, ListOf):
                e = typ.elem
                if isinstance(e, Message):
                    if depth.get(e.name, 0) >= max_depth:
                        continue
                    i = self._add(path, tag, Kind.LIST, Kind.MESSAGE, parent)
                    d2 = dict(depth)
                    d2[e.name] = d2.get(e.name, 0) + 1
                    self._add_message(e, i, path + "[].", d2, max_depth)
                elif isinstance(e, Struct):
                    i = self._add(path, tag, Kind.LIST, Kind.STRUCT, parent)
                    self._add_members(e, i, f"{path}[].")
                else:
                    self._add(path, tag, Kind.LIST, Kind(e), parent)
            elif isinstance(typ, Message):
                if depth.get(typ.name, 0) >= max_depth:
                    continue
                i = self._add(path, tag, Kind.MESSAGE, 0, parent)
                d2 = dict(depth)
                d2[typ.name] = d2.get(typ.name, 0) + 1
                self._add_message(typ, i, path + ".", d2, max_depth)
            elif isinstance(typ, Struct):
                i = self._add(path, tag, Kind.STRUCT, 0, parent)
                self._add_members(typ, i, path + ".")
            else:
                self._add(path, tag, Kind(typ), 0, parent)

    def _add_members(self, struct, parent, prefix):
        """A struct's members in declaration order (pre-order: a struct member's own members
        follow it)."""
        for m, k in struct.members:
            if isinstance(k, Struct):
                j = self._add(prefix + m, 0, Kind.STRUCT, 0, parent)
                self._add_members(k, j, f"{prefix}{m}.")
            else:
                self._add(prefix + m, 0, k, 0, parent)

    # -- layout (spec_tree_layout) --
    def _layout(self):
        T = (_lib.SpecTreeTable * _lib.SPEC_TREE_MAX_TABLES)()
        K = (_lib.SpecTreeColumn * _lib.SPEC_TREE_MAX_COLUMNS)()
        nt, nc = C.c_uint32(0), C.c_uint32(0)
        _lib.check(_lib.lib().spec_tree_layout(C.byref(self.c), T, C.byref(nt), K, C.byref(nc)), "spec_tree_layout")
        self.tables = []
        for x in range(nt.value):
            t = T[x]
            if t.field < 0:
                path = ""
            else:
                f = self.fields[t.field]
                path = f.path + ("[]" if f.kind == Kind.LIST else "")
            self.tables.append(TreeTable(x, path, t.parent, t.field, t.rel, t.shape))
        self.columns = []
        for c in range(nc.value):
            k = K[c]
            tb = self.tables[k.table]
            f = self.fields[k.field] if k.field >= 0 else None
            if k.role == ROLE_BEGIN:
                name = f"{f.path}#begin"
            elif k.role == ROLE_STATUS:
                name = f"{tb.path}#status"
            elif k.role == ROLE_ERRMASK:
                name = f"{tb.path}#errmask"
            elif k.role == ROLE_TYPE:
                name = f"{f.path}#type"
            elif k.role == ROLE_PRESENT:
                name = f"{f.path}?"
            elif f is not None and f.kind == Kind.LIST:  # a value list's elements
                name = f"{f.path}[]"
            else:
                name = f.path
            col = TreeColumn(c, name, k.table, k.field, k.role, k.kind, k.width)
            self.columns.append(col)
            tb.columns.append(col)
        self.by_name = {c.name: c for c in self.columns}

    def column(self, name: str) -> TreeColumn:
        return self.by_name[name]

    def column_rows(self, c: TreeColumn, rows) -> int:
        """Entries of column c given the table row counts (BEGIN: owner rows + 1)."""
        if c.role == ROLE_BEGIN:
            return rows[self.tables[c.table].parent] + 1
        return rows[c.table]

    def span_columns(self):
        return [c for c in self.columns if c.role == ROLE_VALUE and c.kind in (Kind.STRING, Kind.BYTES, Kind.ANY)]


def _stream_handle(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return C.c_void_p(s.cuda_stream)


@dataclass
class TreeColumns:
    tree: Tree
    rows: list
    cols: list  # uint8 [entries, width] device tensors in layout order

    def __getitem__(self, name: str) -> torch.Tensor:
        return self.cols[self.tree.by_name[name].index]

    def numpy(self, name: str) -> np.ndarray:
        c = self.tree.by_name[name]
        a = self.cols[c.index].cpu().numpy()
        if c.role in (ROLE_PRESENT, ROLE_STATUS, ROLE_TYPE):
            return a.reshape(-1)
        if c.role == ROLE_ERRMASK:
            return a.view(np.uint64).reshape(-1)
        if c.role == ROLE_BEGIN:
            return a.view(np.uint32).reshape(-1)
        return a


class TreeDecoder:
    """spec_tree_decoder: index() the batch (row counts per table), then decode() every column."""

    def __init__(self, tree: Tree):
        self.tree = tree
        self._h = C.c_void_p()
        _lib.check(_lib.lib().spec_tree_decoder_create(C.byref(tree.c), C.byref(self._h)), "spec_tree_decoder_create")
        self.rows = None

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and h.value:
            try:
                _lib.lib().spec_tree_decoder_destroy(h)
            except Exception:
                pass

    def index(self, stream: torch.Tensor, ends: torch.Tensor, cuda_stream=None) -> list:
        if not (stream.is_cuda and ends.is_cuda and stream.dtype == torch.uint8 and ends.dtype == torch.int64):
            raise ValueError("stream uint8 and ends int64 device tensors")
        self._keep = (stream, ends)
        rows = (C.c_uint64 * len(self.tree.tables))()
        rc = _lib.lib().spec_tree_decoder_index(self._h, C.c_void_p(stream.data_ptr()), stream.numel(),
                                                 C.c_void_p(ends.data_ptr()), ends.numel(), rows,
                                                 _stream_handle(cuda_stream))
        _lib.check(rc, "spec_tree_decoder_index")
        self.rows = [int(r) for r in rows]
        return self.rows

    def index_spans(self, stream: torch.Tensor, spans: torch.Tensor, cuda_stream=None) -> list:
        """index() over value spans (an `any` / `message` column, int32/uint32 [n, 2] or uint8
        [n, 8]): row i of the root table = m.Field(tag).Message() of record i
        (spec_tree_decoder_index_spans)."""
        if not (stream.is_cuda and spans.is_cuda and stream.dtype == torch.uint8 and spans.is_contiguous()):
            raise ValueError("stream uint8 and contiguous spans device tensors")
        if spans.numel() * spans.element_size() % 8:
            raise ValueError("spans: 8 bytes (off, len) per value")
        n = spans.numel() * spans.element_size() // 8
        self._keep = (stream, spans)
        rows = (C.c_uint64 * len(self.tree.tables))()
        rc = _lib.lib().spec_tree_decoder_index_spans(self._h, C.c_void_p(stream.data_ptr()), stream.numel(),
                                                       C.c_void_p(spans.data_ptr()), n, rows,
                                                       _stream_handle(cuda_stream))
        _lib.check(rc, "spec_tree_decoder_index_spans")
        self.rows = [int(r) for r in rows]
        return self.rows

    def alloc(self, device) -> list:
        return [torch.empty((max(self.tree.column_rows(c, self.rows), 1), c.width), dtype=torch.uint8, device=device)
                for c in self.tree.columns]

    def column_capacity(self, cols: list) -> list:
        """Rows each table's columns hold (the smallest of its columns; a BEGIN column of n + 1
        entries holds n rows of the owner table); None entries do not limit."""
        cap = [None] * len(self.tree.tables)
        for c, tc in zip(cols, self.tree.columns):
            if c is None:
                continue
            entries = c.numel() * c.element_size() // tc.width
            t, k = (self.tree.tables[tc.table].parent, entries - 1) if tc.role == ROLE_BEGIN else (tc.table, entries)
            cap[t] = k if cap[t] is None else min(cap[t], k)
        return [(1 << 64) - 1 if k is None else max(k, 0) for k in cap]

    def capacity(self) -> list:
        """The decoder's list-table row capacities (spec_tree_decoder_capacity)."""
        r = (C.c_uint64 * len(self.tree.tables))()
        _lib.check(_lib.lib().spec_tree_decoder_capacity(self._h, r), "spec_tree_decoder_capacity")
        return [int(x) for x in r]

    def run(self, stream: torch.Tensor, ends: torch.Tensor, cols: list, rows_out: torch.Tensor | None = None,
            cuda_stream=None, col_rows=None) -> torch.Tensor:
        """Decode a new batch into `cols` in one asynchronous pass (spec_tree_decoder_run): no
        host synchronisation; returns the device row counts (int64 [ntables], -1 where a list
        table outgrew the decoder's capacity or its columns, and below such a list: index() a
        batch of that shape first).  Rows are clamped to what `cols` hold: nothing is written
        past a column (`col_rows`: column_capacity(cols), precomputed by a caller that runs
        the same columns repeatedly)."""
        if not (stream.is_cuda and ends.is_cuda and stream.dtype == torch.uint8 and ends.dtype == torch.int64):
            raise ValueError("stream uint8 and ends int64 device tensors")
        if len(cols) != len(self.tree.columns):
            raise ValueError("one entry per column (None skips it)")
        if rows_out is None:
            rows_out = torch.empty(len(self.tree.tables), dtype=torch.int64, device=stream.device)
        self._keep = (stream, ends)
        ptrs = (C.c_void_p * len(cols))(*[c.data_ptr() if c is not None else 0 for c in cols])
        caps = (C.c_uint64 * len(self.tree.tables))(*(col_rows if col_rows is not None else self.column_capacity(cols)))
        rc = _lib.lib().spec_tree_decoder_run(self._h, C.c_void_p(stream.data_ptr()), stream.numel(),
                                               C.c_void_p(ends.data_ptr()), ends.numel(), ptrs, caps,
                                               C.c_void_p(rows_out.data_ptr()), _stream_handle(cuda_stream))
        _lib.check(rc, "spec_tree_decoder_run")
        return rows_out

    def reserve(self, rows):
        """List-table capacities of at least rows[t] (spec_tree_decoder_reserve)."""
        r = (C.c_uint64 * len(self.tree.tables))(*rows)
        _lib.check(_lib.lib().spec_tree_decoder_reserve(self._h, r), "spec_tree_decoder_reserve")

    def decode(self, cols=None, cuda_stream=None) -> TreeColumns:
        if self.rows is None:
            raise RuntimeError("index() first")
        dev = self._keep[0].device
        cols = cols if cols is not None else self.alloc(dev)
        ptrs = (C.c_void_p * len(cols))(*[c.data_ptr() if c is not None else 0 for c in cols])
        rc = _lib.lib().spec_tree_decoder_decode(self._h, ptrs, _stream_handle(cuda_stream))
        _lib.check(rc, "spec_tree_decoder_decode")
        out = [c[: self.tree.column_rows(tc, self.rows)] if c is not None else None
               for c, tc in zip(cols, self.tree.columns)]
        return TreeColumns(self.tree, list(self.rows), out)


def decode_tree(tree: Tree, stream: torch.Tensor, ends: torch.Tensor, cuda_stream=None) -> TreeColumns:
    d = TreeDecoder(tree)
    d.index(stream, ends, cuda_stream)
    return d.decode(cuda_stream=cuda_stream)


def decode_values(kind, stream: torch.Tensor, spans: torch.Tensor, cuda_stream=None):
    """Value.<Kind>() / <Kind>Err() over value spans (an `any` column): -> (values uint8 [n,
    width], err uint8 [n]: 1 decoder error, 2 span past the stream) (spec_decode_values)."""
    kind = Kind(kind)
    if not (stream.is_cuda and spans.is_cuda and stream.dtype == torch.uint8 and spans.is_contiguous()):
        raise ValueError("stream uint8 and contiguous spans device tensors")
    n = spans.numel() * spans.element_size() // 8
    out = torch.empty((max(n, 1), WIDTH[kind]), dtype=torch.uint8, device=stream.device)
    err = torch.empty(max(n, 1), dtype=torch.uint8, device=stream.device)
    rc = _lib.lib().spec_decode_values(int(kind), C.c_void_p(stream.data_ptr()), stream.numel(),
                                       C.c_void_p(spans.data_ptr()), n, C.c_void_p(out.data_ptr()),
                                       C.c_void_p(err.data_ptr()), _stream_handle(cuda_stream))
    _lib.check(rc, "spec_decode_values")
    return out[:n], err[:n]


def tree_rows(tree: Tree, n: int, cols: dict) -> list:
    """Row counts per table from the record count and the BEGIN columns (host reads)."""
    rows = [0] * len(tree.tables)
    rows[0] = n
    for t in tree.tables[1:]:
        if t.rel == REL_ONE:
            rows[t.index] = rows[t.parent]
        else:
            b = cols[f"{tree.fields[t.field].path}#begin"]
            b = b.cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
            rows[t.index] = int(b.reshape(-1).view(np.uint32)[rows[t.parent]]) if rows[t.parent] >= 0 else 0
    return rows


class TreeEncoder:
    """spec_encode_tree: the generated Write() of every record over the tree."""

    def __init__(self, tree: Tree, rows: list, device="cuda"):
        self.tree, self.rows = tree, list(rows)
        self._rows = (C.c_uint64 * len(rows))(*rows)
        ws = _lib.lib().spec_encode_tree_workspace_size(C.byref(tree.c), self._rows)
        self.workspace = torch.empty((ws + 7) // 8, dtype=torch.int64, device=device)
        self.ws_bytes = ws
        self.total = torch.zeros(1, dtype=torch.int64, device=device)

    def _args(self, cols: dict, heaps: dict):
        t = self.tree
        nc = len(t.columns)
        cp = (C.c_void_p * nc)()
        hp = (C.c_void_p * nc)()
        hl = (C.c_uint64 * nc)()
        keep = []
        for c in t.columns:
            v = cols.get(c.name)
            if c.role not in INPUT_ROLES:
                continue  # decode outputs (STATUS, ERRMASK, TYPE): not read by the encoder
            if v is None:
                if t.column_rows(c, self.rows) > 0:
                    raise ValueError(f"missing column {c.name}")
                continue
            if not v.is_cuda or not v.is_contiguous():
                raise ValueError(f"column {c.name} must be a contiguous device tensor")
            if v.numel() * v.element_size() < t.column_rows(c, self.rows) * c.width:
                raise ValueError(f"column {c.name} too small")
            keep.append(v)
            cp[c.index] = v.data_ptr()
            if c.role == ROLE_VALUE and c.kind in (Kind.STRING, Kind.BYTES, Kind.ANY):
                h = heaps.get(c.name)
                if h is None:
                    raise ValueError(f"missing heap for {c.name}")
                if not isinstance(h, torch.Tensor) or h.dtype != torch.uint8 or not h.is_contiguous() \
                        or h.device != v.device:
                    raise ValueError(f"heap {c.name} must be a contiguous uint8 tensor on {v.device}")
                keep.append(h)
                hp[c.index] = h.data_ptr()
                hl[c.index] = h.numel()
        return cp, hp, hl, keep

    def encode(self, cols: dict, heaps: dict, out: torch.Tensor | None, ends: torch.Tensor | None, cuda_stream=None):
        cp, hp, hl, keep = self._args(cols, heaps)
        rc = _lib.lib().spec_encode_tree(C.byref(self.tree.c), cp, hp, hl, self._rows,
                                         C.c_void_p(out.data_ptr() if out is not None else 0),
                                         out.numel() if out is not None else 0,
                                         C.c_void_p(ends.data_ptr() if ends is not None else 0),
                                         C.c_void_p(self.workspace.data_ptr()), self.ws_bytes,
                                         C.c_void_p(self.total.data_ptr()), _stream_handle(cuda_stream))
        _lib.check(rc, "spec_encode_tree")
        return self.total


def encode_tree(tree: Tree, cols: dict, heaps: dict, n: int, rows=None, cuda_stream=None):
    """-> (stream uint8 [total], ends int64 [n]) on the device."""
    rows = rows if rows is not None else tree_rows(tree, n, cols)
    some = next(v for v in cols.values() if v is not None)
    enc = TreeEncoder(tree, rows, some.device)
    total = int(enc.encode(cols, heaps, None, None, cuda_stream).item())
    if total < 0:
        raise _lib.SpecError(-1, "spec_encode_tree: encoder error")
    out = torch.empty(max(total, 1), dtype=torch.uint8, device=some.device)
    ends = torch.empty(max(n, 1), dtype=torch.int64, device=some.device)
    enc.encode(cols, heaps, out, ends, cuda_stream)
    return out[:total], ends[:n]


# ---- pkg1.spec (internal/tests/pkg1/pkg1.spec:9-61, pkg2/submessage.spec, pkg3/pkg3a/struct.spec) ----

def pkg1_message(with_any: bool = True) -> Message:
    """The reference's test object schema `pkg1.Message`, fields in the order pkg1.Object.Write
    writes them (internal/tests/pkg1/object.go:60-179): scalars, enum1, struct1, then message1,
    the sub-messages and the lists.  Message1 is a map[uint16]int32 written as a message (Go map
    order is random); here its TestObject keys 1..3 in order.  Enum -> int32."""
    struct = Struct("Struct", [("key", Kind.INT32), ("value", Kind.INT32)])
    value = Struct("pkg3a.Value", [("x", Kind.INT32), ("y", Kind.INT32)])
    sub = Message("Submessage")
    sub.fields = [("value", 1, Kind.STRING), ("next", 2, sub)]
    sub1 = Message("pkg2.Submessage", [("key", 1, Kind.STRING), ("value", 2, value)])
    message1 = Message("message1", [("f1", 1, Kind.INT32), ("f2", 2, Kind.INT32), ("f3", 3, Kind.INT32)])
    fields = [
        ("bool", 1, Kind.BOOL), ("byte", 2, Kind.BYTE),
        ("int16", 10, Kind.INT16), ("int32", 11, Kind.INT32), ("int64", 12, Kind.INT64),
        ("uint16", 20, Kind.UINT16), ("uint32", 21, Kind.UINT32), ("uint64", 22, Kind.UINT64),
        ("float32", 30, Kind.FLOAT32), ("float64", 31, Kind.FLOAT64),
        ("bin64", 40, Kind.BIN64), ("bin128", 41, Kind.BIN128), ("bin256", 42, Kind.BIN256),
        ("string", 50, Kind.STRING), ("bytes1", 51, Kind.BYTES),
        ("enum1", 60, Kind.INT32), ("struct1", 61, struct), ("message1", 52, message1),
        ("submessage", 62, sub), ("submessage1", 63, sub1),
        ("ints", 70, ListOf(Kind.INT64)), ("strings", 71, ListOf(Kind.STRING)), ("structs", 73, ListOf(struct)),
        ("submessages", 74, ListOf(sub)), ("submessages1", 75, ListOf(sub1)),
    ]
    if with_any:
        fields.append(("any", 80, Kind.ANY))
    return Message("Message", fields)



def pkg1_tree(max_depth: int = 2) -> Tree:
    return Tree(pkg1_message(), max_depth=max_depth)


__all__ = ["Struct", "Message", "ListOf", "Tree", "TreeDecoder", "TreeEncoder", "TreeColumns", "decode_tree",
           "decode_values",
           "encode_tree", "tree_rows", "pkg1_message", "pkg1_tree", "WIDTH"]
