"""Schemas from `.spec` files: the reference's schema language
(internal/lang/parser/grammar.y) parsed into the engine's schema descriptors.

    file        imports options definitions                                  grammar.y:180-188
    imports     import ( ["alias"] "path" ... )                              :192-232
    options     options ( name = "value" ... )                               :241-276
    enum        enum Name { NAME = int; ... }                                :369-407
    message     message Name { field type tag; ... [;] }                     :411-458
    struct      struct Name { field type; ... }                              :461-499
    service     (sub)service Name { method(input) [oneway | output | channel [output]]; }  :502-753
    type        base | [] base; base = ident | pkg.ident | any | message     :281-343
Field, method and argument names may be keywords (any, import, message, options, struct,
service, subservice: grammar.y:138-177).

What the generated code does with a field type (internal/lang/generator/message.go:97-439,
type.go:174-329) decides its descriptor:
    bool ... bytes        the scalar Kind          <Enum>     Kind.INT32 (generator/enum.go:69-92)
    <Struct>              tree.Struct              <Message>  tree.Message (sub-message)
    []<scalar|Struct|Message>  tree.ListOf          any, message   Kind.ANY (a span of the raw
                                                                  value: Field(tag), Field(tag).Message())
`SpecSet.tree(name)` gives the spec_amd.Tree of a message (any shape);
`SpecFile.schema(name)` the flat Schema / NestedSchema of the benchmark kernels where one exists.
"""
from __future__ import annotations

import os
import re

from .schema import Field, Kind, NestedSchema, Schema

SCALARS = {
    "bool": Kind.BOOL, "byte": Kind.BYTE, "int16": Kind.INT16, "int32": Kind.INT32, "int64": Kind.INT64,
    "uint16": Kind.UINT16, "uint32": Kind.UINT32, "uint64": Kind.UINT64, "float32": Kind.FLOAT32,
    "float64": Kind.FLOAT64, "bin64": Kind.BIN64, "bin128": Kind.BIN128, "bin256": Kind.BIN256,
    "string": Kind.STRING, "bytes": Kind.BYTES,
}
KEYWORDS = ("any", "enum", "import", "message", "oneway", "options", "struct", "service", "subservice")

_TOKEN = re.compile(r'\s*(//[^\n]*|/\*.*?\*/|"(?:[^"\\]|\\.)*"|[A-Za-z_][A-Za-z0-9_]*|-?\d+|->|<-|[{}()\[\];=,.<>-])',
                    re.S)


def _tokens(text):
    pos, out = 0, []
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m:
            if text[pos:].strip() == "":
                break
            line = text.count("\n", 0, pos) + 1
            raise SyntaxError(f"spec:{line}: unexpected input {text[pos:pos + 20]!r}")
        pos = m.end()
        t = m.group(1)
        if not t.startswith("//") and not t.startswith("/*"):
            out.append(t)
    return out


class SpecFile:
    """One parsed .spec file: imports {alias: path}, options, enums {name: {value: int}},
    messages {name: [(field, type, tag)]}, structs {name: [(field, type)]}, services
    {name: [(method, input, output, oneway, channel)]}; types are strings ("int64",
    "[]pkg1.Struct", "any", "message")."""

    def __init__(self, text: str, package: str = ""):
        self.imports, self.options = {}, {}
        self.enums, self.messages, self.structs, self.services = {}, {}, {}, {}
        self._t = _tokens(text)
        self._i = 0
        self._file()
        gp = self.options.get("go_package", "")
        self.package = package or (gp.rsplit("/", 1)[-1] if gp else "")

    # ---- token helpers ----
    def _peek(self, k=0):
        j = self._i + k
        return self._t[j] if j < len(self._t) else None

    def _next(self):
        t = self._peek()
        if t is None:
            raise SyntaxError("spec: unexpected end of file")
        self._i += 1
        return t

    def _expect(self, t):
        got = self._next()
        if got != t:
            raise SyntaxError(f"spec: expected {t!r}, got {got!r} (token {self._i})")

    def _ident(self):
        t = self._next()
        if not re.match(r"[A-Za-z_]", t):
            raise SyntaxError(f"spec: expected a name, got {t!r}")
        return t

    def _int(self):
        t = self._next()
        if not re.fullmatch(r"-?\d+", t):
            raise SyntaxError(f"spec: expected an integer, got {t!r}")
        return int(t)

    # ---- grammar ----
    def _file(self):
        if self._peek() == "import":
            self._next()
            self._expect("(")
            while self._peek() != ")":
                t = self._next()
                if t.startswith('"'):
                    path = t[1:-1]
                    self.imports[path.rsplit("/", 1)[-1]] = path
                else:  # alias "path"
                    path = self._next()[1:-1]
                    self.imports[t] = path
            self._next()
        if self._peek() == "options":
            self._next()
            self._expect("(")
            while self._peek() != ")":
                name = self._ident()
                self._expect("=")
                self.options[name] = self._next()[1:-1]
            self._next()
        while self._peek() is not None:
            kw = self._next()
            if kw == "enum":
                self._enum()
            elif kw == "message":
                self._message()
            elif kw == "struct":
                self._struct()
            elif kw in ("service", "subservice"):
                self._service()
            else:
                raise SyntaxError(f"spec: unexpected {kw!r}")

    def _type(self):
        if self._peek() == "[":
            self._next()
            self._expect("]")
            return "[]" + self._base_type()
        return self._base_type()

    def _base_type(self):
        t = self._ident()
        if self._peek() == ".":
            self._next()
            t = t + "." + self._ident()
        return t

    def _enum(self):
        name = self._ident()
        self._expect("{")
        vals = {}
        while self._peek() != "}":
            v = self._ident()
            self._expect("=")
            vals[v] = self._int()
            self._expect(";")
        self._next()
        self.enums[name] = vals

    def _message(self):
        name = self._ident()
        self._expect("{")
        fields = []
        while self._peek() != "}":
            if self._peek() == ";":  # semi_opt / separators
                self._next()
                continue
            fname = self._ident()
            typ = self._type()
            fields.append((fname, typ, self._int()))
        self._next()
        self.messages[name] = fields

    def _struct(self):
        name = self._ident()
        self._expect("{")
        fields = []
        while self._peek() != "}":
            fname = self._ident()
            typ = self._type()
            self._expect(";")
            fields.append((fname, typ))
        self._next()
        self.structs[name] = fields

    def _field_list(self):
        """'(' [base_type | method_field, ...] ')' -> a type name or [(name, type, tag)]."""
        self._expect("(")
        if self._peek() == ")":
            self._next()
            return []
        if self._peek(1) in (")", "."):  # a single base type: (Request) / (pkg.Request)
            t = self._base_type()
            self._expect(")")
            return t
        out = []
        while self._peek() != ")":
            if self._peek() == ",":
                self._next()
                continue
            fname = self._ident()
            typ = self._type()
            out.append((fname, typ, self._int()))
        self._next()
        return out

    def _channel(self):
        """'(' [<-In | In<-] [, Out-> | ->Out] ')' (grammar.y:645-709) -> {'in': t, 'out': t}"""
        self._expect("(")
        ch = {}
        while self._peek() != ")":
            t = self._peek()
            if t == ",":
                self._next()
            elif t == "<-":
                self._next()
                ch["in"] = self._type()
            elif t == "->":
                self._next()
                ch["out"] = self._type()
            else:
                typ = self._type()
                arrow = self._next()
                ch["in" if arrow == "<-" else "out"] = typ
        self._next()
        return ch

    def _service(self):
        name = self._ident()
        self._expect("{")
        methods = []
        while self._peek() != "}":
            mname = self._ident()
            inp = self._field_list()
            out, oneway, channel = None, False, None
            if self._peek() == "oneway":
                self._next()
                oneway = True
            elif self._peek() == "(":
                # a channel starts with '<-' or a type followed by '<-' / '->' (or '->' type)
                j = self._i + 1
                is_channel = self._t[j] in ("<-", "->") or any(self._t[k] in ("<-", "->") for k in range(j, j + 4)
                                                               if k < len(self._t) and self._t[k] != ")")
                if is_channel:
                    channel = self._channel()
                    if self._peek() != ";":
                        out = self._field_list() if self._peek() == "(" else self._base_type()
                else:
                    out = self._field_list()
            elif self._peek() != ";":
                out = self._base_type()
            self._expect(";")
            methods.append((mname, inp, out, oneway, channel))
        self._next()
        self.services[name] = methods

    # ---- descriptors ----
    def _kind(self, typ):
        if typ in SCALARS:
            return SCALARS[typ]
        if typ in self.enums:
            return Kind.INT32
        return None

    def schema(self, name: str, skip_unsupported: bool = False):
        """Schema (flat message) or NestedSchema (one []Message field) of message `name`, for the
        schema-specialised flat / nested kernels."""
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
                raise ValueError(f"spec: {name}.{fname}: type {typ} has no flat/nested kind (use SpecSet.tree)")
        return NestedSchema(fields, list(item.fields)) if item is not None else Schema(fields)


class SpecSet:
    """Parsed .spec files by package (the import path's last element, as the generator names
    them), with cross-package type references (`pkg2.Submessage`) resolved."""

    def __init__(self):
        self.files = {}  # package -> SpecFile (a package may span several files: merged)

    def add(self, sf: SpecFile):
        cur = self.files.get(sf.package)
        if cur is None:
            self.files[sf.package] = sf
            return sf
        for attr in ("enums", "messages", "structs", "services", "imports"):
            getattr(cur, attr).update(getattr(sf, attr))
        return cur

    def _lookup(self, pkg: str, typ: str):
        """-> ('enum'|'message'|'struct', package, name)"""
        if "." in typ:
            alias, typ = typ.split(".", 1)
            f = self.files[pkg]
            path = f.imports.get(alias, alias)
            pkg = path.rsplit("/", 1)[-1]
        f = self.files[pkg]
        for kind, table in (("enum", f.enums), ("message", f.messages), ("struct", f.structs)):
            if typ in table:
                return kind, pkg, typ
        raise KeyError(f"spec: unknown type {typ!r} in package {pkg!r}")

    def message(self, name: str, package: str = None, _cache=None):
        """tree.Message of message `name` (recursive references share one object)."""
        from .tree import ListOf, Message, Struct

        cache = _cache if _cache is not None else {}
        pkg = package if package is not None else next(iter(self.files))
        key = (pkg, name)
        if key in cache:
            return cache[key]
        msg = Message(f"{pkg}.{name}" if pkg else name)
        cache[key] = msg

        def resolve(typ):
            if typ in SCALARS:
                return SCALARS[typ]
            if typ in ("any", "message"):
                return Kind.ANY
            kind, p, n = self._lookup(pkg, typ)
            if kind == "enum":
                return Kind.INT32
            if kind == "struct":
                return self.struct(n, p)
            return self.message(n, p, cache)

        fields = []
        for fname, typ, tag in self.files[pkg].messages[name]:
            if typ.startswith("[]"):
                fields.append((fname, tag, ListOf(resolve(typ[2:]))))
            else:
                fields.append((fname, tag, resolve(typ)))
        msg.fields = fields
        return msg

    def struct(self, name: str, package: str, _seen=()):
        """tree.Struct of struct `name`: members are value types (scalars, enums) or other structs
        (internal/lang/model/struct_field.go:57-70); a struct that contains itself is an error."""
        from .tree import Struct

        if (package, name) in _seen:
            raise ValueError(f"spec: struct {name} contains itself")
        members = []
        for mname, mtyp in self.files[package].structs[name]:
            mk = self.scalar_kind(package, mtyp)
            if mk is None:
                kind, p, n = self._lookup(package, mtyp)
                if kind != "struct":
                    raise ValueError(f"spec: struct {name}.{mname}: structs support only value types or other structs")
                mk = self.struct(n, p, _seen + ((package, name),))
            members.append((mname, mk))
        return Struct(f"{package}.{name}", members)

    def scalar_kind(self, pkg, typ):
        """Kind of a scalar or enum type name in package pkg, else None."""
        if typ in SCALARS:
            return SCALARS[typ]
        kind, _, _ = self._lookup(pkg, typ)
        return Kind.INT32 if kind == "enum" else None

    def tree(self, name: str, package: str = None, max_depth: int = 2):
        from .tree import Tree

        return Tree(self.message(name, package), max_depth=max_depth)


def load(text: str, package: str = "") -> SpecFile:
    return SpecFile(text, package)


def load_files(paths, root: str | None = None) -> SpecSet:
    """Parse .spec files into a SpecSet; a file's package = its directory relative to `root`
    (the import path, e.g. "pkg3/pkg3a"), last element, unless options name go_package."""
    s = SpecSet()
    for p in paths:
        text = open(p).read()
        pkg = ""
        if root is not None:
            pkg = os.path.relpath(os.path.dirname(p), root).replace(os.sep, "/").rsplit("/", 1)[-1]
        sf = SpecFile(text, pkg)
        s.add(sf)
    return s
