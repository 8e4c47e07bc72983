"""Tiny reader for the Go composite literals found in the reference's test tables
(text only; used by make_golden.py in the build container).

Values are returned as tagged tuples so int / float64 typing survives:
  ("int", "8") ("float", "8.0") ("str", s) ("bool", b) ("nil",) ("map", {k: v})
  ("list", [v]) ("struct", {field: v}) ("ident", "operator.Equal") ("bytes", s)
"""
import json
import re


class Unsupported(Exception):
    pass


_NUM = re.compile(r"[-+]?(?:\d[\d_]*(?:\.\d*)?|\.\d+)(?:[eE][-+]?\d+)?")
_IDENT = re.compile(r"[A-Za-z_][A-Za-z0-9_.]*")


class Reader:
    def __init__(self, s, i=0):
        self.s, self.i = s, i

    def ws(self):
        s = self.s
        while self.i < len(s):
            if s[self.i] in " \t\r\n":
                self.i += 1
            elif s.startswith("//", self.i):
                j = s.find("\n", self.i)
                self.i = len(s) if j < 0 else j + 1
            else:
                break

    def peek(self, lit):
        self.ws()
        return self.s.startswith(lit, self.i)

    def eat(self, lit):
        if not self.peek(lit):
            raise Unsupported(f"expected {lit!r} at {self.s[self.i:self.i + 40]!r}")
        self.i += len(lit)

    def string(self):
        s = self.s
        if s[self.i] == "`":
            j = s.index("`", self.i + 1)
            out = s[self.i + 1:j]
            self.i = j + 1
            return out
        j = self.i + 1
        out = []
        while s[j] != '"':
            c = s[j]
            if c == "\\":
                n = s[j + 1]
                m = {"n": "\n", "t": "\t", "r": "\r", '"': '"', "\\": "\\", "'": "'", "a": "\a", "b": "\b",
                     "f": "\f", "v": "\v"}
                if n in m:
                    out.append(m[n])
                    j += 2
                elif n == "u":
                    out.append(chr(int(s[j + 2:j + 6], 16)))
                    j += 6
                elif n == "x":
                    out.append(chr(int(s[j + 2:j + 4], 16)))
                    j += 4
                else:
                    raise Unsupported("escape")
            else:
                out.append(c)
                j += 1
        self.i = j + 1
        return "".join(out)

    def fields(self, close="}"):
        """key: value pairs (struct or map literal body) up to the closing brace."""
        out = {}
        while True:
            self.ws()
            if self.peek(close):
                self.i += 1
                return out
            if self.s[self.i] in "\"`":
                k = self.string()
            else:
                m = _IDENT.match(self.s, self.i)
                if not m:
                    raise Unsupported("field name")
                k = m.group(0)
                self.i = m.end()
            self.eat(":")
            out[k] = self.value()
            self.ws()
            if self.peek(","):
                self.i += 1

    def elements(self, close="}"):
        out = []
        while True:
            self.ws()
            if self.peek(close):
                self.i += 1
                return out
            out.append(self.value())
            self.ws()
            if self.peek(","):
                self.i += 1

    def value(self):
        self.ws()
        s, i = self.s, self.i
        if s[i] in "\"`":
            return ("str", self.string())
        for kw, v in (("nil", ("nil",)), ("true", ("bool", True)), ("false", ("bool", False))):
            if s.startswith(kw, i) and not (s[i + len(kw):i + len(kw) + 1].isalnum()):
                self.i += len(kw)
                return v
        for pre in ("map[string]interface{}(nil)",):
            if s.startswith(pre, i):
                self.i += len(pre)
                return ("map", {})
        if s.startswith("map[string]interface{}{", i):
            self.i += len("map[string]interface{}{")
            return ("map", self.fields())
        if s.startswith("[]interface{}{", i):
            self.i += len("[]interface{}{")
            return ("list", self.elements())
        if s.startswith("[]byte(", i):
            self.i += len("[]byte(")
            self.ws()
            v = self.string()
            self.eat(")")
            return ("bytes", v)
        for conv, tag in (("int64(", "int"), ("int(", "int"), ("float64(", "float")):
            if s.startswith(conv, i):
                self.i += len(conv)
                v = self.value()
                self.eat(")")
                if v[0] not in ("int", "float"):
                    raise Unsupported("conversion")
                if tag == "float" and v[0] == "int":
                    return ("float", v[1] + ".0")
                if tag == "int" and v[0] == "float":
                    raise Unsupported("float->int conversion")
                return v
        if s[i] == "{":
            self.i += 1
            return ("struct", self.fields())
        m = re.match(r"(\[\][\w.]+|map\[[\w.]+\][\w.{}]+?)(\{|\(nil\))", s[i:i + 80])
        if m:  # other composite literal types: kept opaque (to_json rejects them)
            self.i += m.end()
            if m.group(2) == "(nil)":
                return ("other", None)
            body = self.elements() if m.group(1).startswith("[]") else self.fields()
            return ("other", body)
        m = _NUM.match(s, i)
        if m and m.group(0) not in ("+", "-"):
            t = m.group(0).replace("_", "")
            self.i = m.end()
            return ("float" if any(c in t for c in ".eE") else "int", t)
        m = _IDENT.match(s, i)
        if m:
            self.i = m.end()
            name = m.group(0)
            self.ws()
            if self.peek("{"):
                self.i += 1
                return ("struct", self.fields())
            return ("ident", name)
        raise Unsupported(f"value at {s[i:i + 30]!r}")


def to_json(v):
    """Tagged value -> JSON text (integer literals stay integers, floats keep a '.')."""
    t = v[0]
    if t == "int":
        return str(int(v[1]))
    if t == "float":
        x = v[1]
        if x.startswith("+"):
            x = x[1:]
        if x.startswith("."):
            x = "0" + x
        if x.startswith("-."):
            x = "-0" + x[1:]
        if x.endswith("."):
            x += "0"
        return x
    if t == "str":
        return json.dumps(v[1])
    if t == "bool":
        return "true" if v[1] else "false"
    if t == "nil":
        return "null"
    if t == "map":
        return "{" + ",".join(json.dumps(k) + ":" + to_json(x) for k, x in v[1].items()) + "}"
    if t == "list":
        return "[" + ",".join(to_json(x) for x in v[1]) + "]"
    raise Unsupported(t)


def table(text, func):
    """Cases (list of tagged structs) of `tests := []struct{...}{...}` inside func."""
    i = text.index(f"func {func}(")
    j = text.index("[]struct", i)
    k = text.index("{", j)
    depth = 0
    while True:  # skip the struct type body
        if text[k] == "{":
            depth += 1
        elif text[k] == "}":
            depth -= 1
            if depth == 0:
                break
        k += 1
    r = Reader(text, k + 1)
    r.eat("{")
    return r.elements()
