"""protoc-lite: a minimal proto3 front end.

There is no ``protoc``/``grpc_tools`` on the MI355X image, and the reference
ships generated ``*_pb2.py`` files produced at build time from an external repo
(reference ``src/python/library/build_wheel.py:126-153``).  Instead we parse the
authored ``.proto`` text directly into ``FileDescriptorProto`` messages and hand
them to the protobuf runtime's descriptor pool.  The same parse tree drives the
C++ code generator (``tools/gen_cpp_proto.py``), so Python and C++ cannot drift.

Supported: ``syntax``, ``package``, ``import``, ``option`` (ignored),
``message`` / ``enum`` (nested), ``repeated`` / ``optional`` fields,
``map<K,V>``, ``oneof``, ``reserved`` (ignored), ``service`` with (client/server
streaming) ``rpc``.
"""

import os
import re

from google.protobuf import descriptor_pb2

_FDP = descriptor_pb2.FieldDescriptorProto

SCALARS = {
    "double": _FDP.TYPE_DOUBLE,
    "float": _FDP.TYPE_FLOAT,
    "int64": _FDP.TYPE_INT64,
    "uint64": _FDP.TYPE_UINT64,
    "int32": _FDP.TYPE_INT32,
    "fixed64": _FDP.TYPE_FIXED64,
    "fixed32": _FDP.TYPE_FIXED32,
    "bool": _FDP.TYPE_BOOL,
    "string": _FDP.TYPE_STRING,
    "bytes": _FDP.TYPE_BYTES,
    "uint32": _FDP.TYPE_UINT32,
    "sfixed32": _FDP.TYPE_SFIXED32,
    "sfixed64": _FDP.TYPE_SFIXED64,
    "sint32": _FDP.TYPE_SINT32,
    "sint64": _FDP.TYPE_SINT64,
}

_TOKEN_RE = re.compile(
    r'\s+|//[^\n]*|/\*.*?\*/|"(?:[^"\\]|\\.)*"|[A-Za-z_][A-Za-z0-9_.]*|-?\d+|[{}()<>;=,\[\]]',
    re.S,
)


def _tokenize(text):
    pos = 0
    out = []
    while pos < len(text):
        m = _TOKEN_RE.match(text, pos)
        if not m:
            raise SyntaxError("proto: unexpected character %r at %d" % (text[pos], pos))
        tok = m.group(0)
        pos = m.end()
        if tok.isspace() or tok.startswith("//") or tok.startswith("/*"):
            continue
        out.append(tok)
    return out


class _Parser:
    def __init__(self, tokens):
        self.t = tokens
        self.i = 0

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def next(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, tok):
        got = self.next()
        if got != tok:
            raise SyntaxError("proto: expected %r got %r (token %d)" % (tok, got, self.i))

    def skip_statement(self):
        depth = 0
        while True:
            tok = self.next()
            if tok == "{":
                depth += 1
            elif tok == "}":
                depth -= 1
                if depth == 0:
                    return
            elif tok == ";" and depth == 0:
                return

    def skip_field_options(self):
        if self.peek() == "[":
            while self.next() != "]":
                pass


# --- AST ------------------------------------------------------------------
class Field:
    def __init__(self, name, number, type_name, label, oneof=None, map_kv=None):
        self.name = name
        self.number = number
        self.type_name = type_name  # scalar name or (unresolved) message/enum name
        self.label = label  # "optional" | "repeated"
        self.oneof = oneof
        self.map_kv = map_kv  # (key_type, value_type) for map fields
        self.resolved = None  # fully-qualified ".pkg.Msg" for message/enum
        self.kind = None  # "scalar" | "message" | "enum"


class Message:
    def __init__(self, name, fqn):
        self.name = name
        self.fqn = fqn
        self.fields = []
        self.oneofs = []
        self.messages = []
        self.enums = []
        self.map_entry = False


class Enum:
    def __init__(self, name, fqn):
        self.name = name
        self.fqn = fqn
        self.values = []


class Rpc:
    def __init__(self, name, input_type, output_type, client_streaming, server_streaming):
        self.name = name
        self.input_type = input_type
        self.output_type = output_type
        self.client_streaming = client_streaming
        self.server_streaming = server_streaming


class Service:
    def __init__(self, name):
        self.name = name
        self.rpcs = []


class ProtoFile:
    def __init__(self, name):
        self.name = name
        self.package = ""
        self.imports = []
        self.messages = []
        self.enums = []
        self.services = []


def _camel(name):
    return "".join(p[:1].upper() + p[1:] for p in name.split("_"))


def parse(text, name):
    p = _Parser(_tokenize(text))
    pf = ProtoFile(name)
    while p.peek() is not None:
        tok = p.next()
        if tok == "syntax":
            p.expect("=")
            if p.next().strip('"') != "proto3":
                raise SyntaxError("protoc-lite only supports proto3")
            p.expect(";")
        elif tok == "package":
            pf.package = p.next()
            p.expect(";")
        elif tok == "import":
            pf.imports.append(p.next().strip('"'))
            p.expect(";")
        elif tok == "option":
            p.skip_statement()
        elif tok == "message":
            pf.messages.append(_parse_message(p, "." + pf.package if pf.package else ""))
        elif tok == "enum":
            pf.enums.append(_parse_enum(p, "." + pf.package if pf.package else ""))
        elif tok == "service":
            pf.services.append(_parse_service(p))
        elif tok == ";":
            continue
        else:
            raise SyntaxError("proto: unexpected top-level token %r" % tok)
    return pf


def _parse_enum(p, scope):
    name = p.next()
    e = Enum(name, scope + "." + name)
    p.expect("{")
    while p.peek() != "}":
        tok = p.next()
        if tok in ("option", "reserved"):
            p.skip_statement()
            continue
        p.expect("=")
        e.values.append((tok, int(p.next())))
        p.skip_field_options()
        p.expect(";")
    p.expect("}")
    return e


def _parse_message(p, scope):
    name = p.next()
    m = Message(name, scope + "." + name)
    p.expect("{")
    _parse_message_body(p, m, None)
    p.expect("}")
    return m


def _parse_field(p, m, first, oneof):
    label = "optional"
    if first in ("repeated", "optional"):
        label = first
        first = p.next()
    if first == "map":
        p.expect("<")
        kt = p.next()
        p.expect(",")
        vt = p.next()
        p.expect(">")
        fname = p.next()
        p.expect("=")
        num = int(p.next())
        p.skip_field_options()
        p.expect(";")
        entry = Message(_camel(fname) + "Entry", m.fqn + "." + _camel(fname) + "Entry")
        entry.map_entry = True
        entry.fields.append(Field("key", 1, kt, "optional"))
        entry.fields.append(Field("value", 2, vt, "optional"))
        m.messages.append(entry)
        f = Field(fname, num, entry.name, "repeated", map_kv=(kt, vt))
        m.fields.append(f)
        return
    fname = p.next()
    p.expect("=")
    num = int(p.next())
    p.skip_field_options()
    p.expect(";")
    m.fields.append(Field(fname, num, first, label, oneof=oneof))


def _parse_message_body(p, m, oneof):
    while p.peek() != "}":
        tok = p.next()
        if tok == "message":
            m.messages.append(_parse_message(p, m.fqn))
        elif tok == "enum":
            m.enums.append(_parse_enum(p, m.fqn))
        elif tok == "oneof":
            oname = p.next()
            m.oneofs.append(oname)
            p.expect("{")
            while p.peek() != "}":
                t2 = p.next()
                if t2 == "option":
                    p.skip_statement()
                    continue
                _parse_field(p, m, t2, len(m.oneofs) - 1)
            p.expect("}")
        elif tok in ("option", "reserved", "extensions"):
            p.skip_statement()
        elif tok == ";":
            continue
        else:
            _parse_field(p, m, tok, oneof)


def _parse_service(p):
    s = Service(p.next())
    p.expect("{")
    while p.peek() != "}":
        tok = p.next()
        if tok == "option":
            p.skip_statement()
            continue
        if tok != "rpc":
            raise SyntaxError("proto: expected rpc, got %r" % tok)
        name = p.next()
        p.expect("(")
        cs = False
        t = p.next()
        if t == "stream":
            cs = True
            t = p.next()
        in_t = t
        p.expect(")")
        p.expect("returns")
        p.expect("(")
        ss = False
        t = p.next()
        if t == "stream":
            ss = True
            t = p.next()
        out_t = t
        p.expect(")")
        if p.peek() == "{":
            p.next()
            while p.next() != "}":
                pass
            if p.peek() == ";":
                p.next()
        else:
            p.expect(";")
        s.rpcs.append(Rpc(name, in_t, out_t, cs, ss))
    p.expect("}")
    return s


# --- resolution -----------------------------------------------------------
def _collect(pf, table):
    def walk_msg(msg):
        table[msg.fqn] = ("message", msg)
        for sub in msg.messages:
            walk_msg(sub)
        for e in msg.enums:
            table[e.fqn] = ("enum", e)

    for msg in pf.messages:
        walk_msg(msg)
    for e in pf.enums:
        table[e.fqn] = ("enum", e)


def _resolve_name(name, scope, table):
    if name.startswith("."):
        return name if name in table else None
    parts = scope.split(".")
    while True:
        cand = ".".join(parts + [name]) if parts != [""] else "." + name
        if not cand.startswith("."):
            cand = "." + cand
        if cand in table:
            return cand
        if not parts or parts == [""]:
            return None
        parts = parts[:-1]


def resolve(files):
    """Resolve every non-scalar field / rpc type across ``files``."""
    table = {}
    for pf in files:
        _collect(pf, table)

    def walk(msg):
        for f in msg.fields:
            if f.type_name in SCALARS:
                f.kind = "scalar"
            else:
                fq = _resolve_name(f.type_name, msg.fqn, table)
                if fq is None:
                    raise SyntaxError("proto: unresolved type %s in %s" % (f.type_name, msg.fqn))
                f.resolved = fq
                f.kind = table[fq][0]
        for sub in msg.messages:
            walk(sub)

    for pf in files:
        for msg in pf.messages:
            walk(msg)
        pkg_scope = "." + pf.package if pf.package else ""
        for s in pf.services:
            for r in s.rpcs:
                r.input_type = _resolve_name(r.input_type, pkg_scope, table)
                r.output_type = _resolve_name(r.output_type, pkg_scope, table)
    return table


# --- FileDescriptorProto emission -----------------------------------------
def _emit_msg(msg, dp):
    dp.name = msg.name
    if msg.map_entry:
        dp.options.map_entry = True
    for o in msg.oneofs:
        dp.oneof_decl.add(name=o)
    for f in msg.fields:
        fd = dp.field.add(name=f.name, number=f.number, json_name=_json_name(f.name))
        fd.label = _FDP.LABEL_REPEATED if f.label == "repeated" else _FDP.LABEL_OPTIONAL
        if f.kind == "scalar":
            fd.type = SCALARS[f.type_name]
        elif f.kind == "enum":
            fd.type = _FDP.TYPE_ENUM
            fd.type_name = f.resolved
        else:
            fd.type = _FDP.TYPE_MESSAGE
            fd.type_name = f.resolved
        if f.oneof is not None:
            fd.oneof_index = f.oneof
    for sub in msg.messages:
        _emit_msg(sub, dp.nested_type.add())
    for e in msg.enums:
        _emit_enum(e, dp.enum_type.add())


def _emit_enum(e, ep):
    ep.name = e.name
    for n, v in e.values:
        ep.value.add(name=n, number=v)


def _json_name(name):
    parts = name.split("_")
    return parts[0] + "".join(x[:1].upper() + x[1:] for x in parts[1:])


def to_file_descriptor_proto(pf):
    fdp = descriptor_pb2.FileDescriptorProto(name=pf.name, package=pf.package, syntax="proto3")
    fdp.dependency.extend(pf.imports)
    for msg in pf.messages:
        _emit_msg(msg, fdp.message_type.add())
    for e in pf.enums:
        _emit_enum(e, fdp.enum_type.add())
    for s in pf.services:
        sp = fdp.service.add(name=s.name)
        for r in s.rpcs:
            mp = sp.method.add(name=r.name, input_type=r.input_type, output_type=r.output_type)
            if r.client_streaming:
                mp.client_streaming = True
            if r.server_streaming:
                mp.server_streaming = True
    return fdp


PROTO_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "proto")


def load_files(names=("model_config.proto", "grpc_service.proto"), proto_dir=PROTO_DIR):
    """Parse + resolve the named .proto files (dependency order)."""
    files = []
    for n in names:
        with open(os.path.join(proto_dir, n)) as f:
            files.append(parse(f.read(), n))
    resolve(files)
    return files
