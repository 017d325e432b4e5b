"""Schema descriptors from `.spec` files.

The reference's code generator turns a `.spec` message into a reader whose getters call one
typed accessor per field (internal/lang/generator/message.go:97-186) and a writer that calls
one FieldWriter method per field in declaration order (message.go:319-439).  `load` parses the
subset of the language those batch kernels cover and returns, per message, the `Schema` (or
`NestedSchema`) the engine decodes/encodes with — the same field order and kinds the generated
code uses:

    bool byte int16 int32 int64 uint16 uint32 uint64 float32 float64 bin64 bin128 bin256
    string bytes   -> the matching Kind
    <Enum>         -> Kind.INT32 (enums are Int32 on the wire, generator/enum.go:69-92)
    []<Message>    -> Kind.LIST with the item message's schema (NestedSchema, one per message)

Other field types (nested messages, structs, lists of scalars, any) have no column kind here:
`load(..., skip_unsupported=True)` leaves them out of the schema (decoding by tag simply does
not read them), otherwise they raise.
"""
from __future__ import annotations

import re

from .schema import Field, Kind, NestedSchema, Schema

SCALARS = {
    "bool": Kind.BOOL, "byte": Kind.BYTE, "int16": Kind.INT16, "int32": Kind.INT32, "int64": Kind.INT64,
    "uint16": Kind.UINT16, "uint32": Kind.UINT32, "uint64": Kind.UINT64, "float32": Kind.FLOAT32,
    "float64": Kind.FLOAT64, "bin64": Kind.BIN64, "bin128": Kind.BIN128, "bin256": Kind.BIN256,
    "string": Kind.STRING, "bytes": Kind.BYTES,
}

_TOKEN = re.compile(r'\s*(//[^\n]*|"[^"]*"|\[\]|[A-Za-z_][A-Za-z0-9_.]*|-?\d+|[{}();=,])')


def _tokens(text):
    pos, out = 0, []
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            if text[pos:].strip() == "":
                break
            raise SyntaxError(f"spec: unexpected input at {text[pos:pos + 20]!r}")
        pos = m.end()
        t = m.group(1)
        if not t.startswith("//"):
            out.append(t)
    return out


class SpecFile:
    """Parsed definitions: enums {name: {value name: int}}, messages/structs {name: [(field, type, tag)]}."""

    def __init__(self, text: str):
        self.enums, self.messages, self.structs = {}, {}, {}
        toks = _tokens(text)
        i = 0

        def expect(t):
            nonlocal i
            if toks[i] != t:
                raise SyntaxError(f"spec: expected {t!r}, got {toks[i]!r}")
            i += 1

        while i < len(toks):
            kw = toks[i]
            if kw in ("import", "options"):
                i += 1
                expect("(")
                while toks[i] != ")":
                    i += 1
                i += 1
            elif kw == "enum":
                name = toks[i + 1]
                i += 2
                expect("{")
                vals = {}
                while toks[i] != "}":
                    vals[toks[i]] = int(toks[i + 2])
                    i += 3
                    expect(";")
                i += 1
                self.enums[name] = vals
            elif kw in ("message", "struct"):
                name = toks[i + 1]
                i += 2
                expect("{")
                fields = []
                while toks[i] != "}":
                    fname = toks[i]
                    i += 1
                    typ = toks[i]
                    i += 1
                    if typ == "[]":
                        typ = "[]" + toks[i]
                        i += 1
                    tag = None
                    if kw == "message":
                        tag = int(toks[i])
                        i += 1
                    expect(";")
                    fields.append((fname, typ, tag))
                i += 1
                (self.messages if kw == "message" else self.structs)[name] = fields
            elif kw == "service":
                depth = 0
                while True:
                    if toks[i] == "{":
                        depth += 1
                    elif toks[i] == "}":
                        depth -= 1
                        if depth == 0:
                            i += 1
                            break
                    i += 1
            else:
                raise SyntaxError(f"spec: unexpected {kw!r}")

    def _kind(self, typ):
        if typ in SCALARS:
            return SCALARS[typ]
        if typ in self.enums:
            return Kind.INT32
        return None

    def schema(self, name: str, skip_unsupported: bool = False):
        """Schema (flat message) or NestedSchema (one []Message field) of message `name`."""
        fields, item = [], None
        for fname, typ, tag in self.messages[name]:
            k = self._kind(typ)
            if k is not None:
                fields.append(Field(tag, k, fname))
            elif typ.startswith("[]") and typ[2:] in self.messages and item is None:
                item = self.schema(typ[2:], skip_unsupported)
                if isinstance(item, NestedSchema):
                    raise ValueError(f"spec: {name}.{fname}: nested lists of lists are not a batch kind")
                fields.append(Field(tag, Kind.LIST, fname))
            elif not skip_unsupported:
                raise ValueError(f"spec: {name}.{fname}: type {typ} has no batch column kind")
        return NestedSchema(fields, list(item.fields)) if item is not None else Schema(fields)


def load(text: str) -> SpecFile:
    return SpecFile(text)
