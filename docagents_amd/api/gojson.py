"""Go ``encoding/json`` compatible writer (the wire format of internal/httputil/httputil.go:37-43).

``json.NewEncoder(w).SetIndent("", "  ").Encode(v)``: maps with sorted keys, 2-space indent,
``": "`` separators, trailing newline, HTML-unsafe characters escaped (``<``, ``>``, ``&``,
U+2028, U+2029), float32 values in Go's shortest float32 representation (``strconv.FormatFloat(f,
'f' or 'e', -1, 32)`` per encoding/json's floatEncoder rules), nil slices as ``null``.
"""
from __future__ import annotations

import math
import re
import struct
from json.encoder import encode_basestring as _encode_basestring

import numpy as _np

_SURR = re.compile("[\ud800-\udfff]")


class F32(float):
    """Marks a value that Go holds as float32 (confidence, score)."""


class Struct(dict):
    """A Go struct: fields encoded in declaration (insertion) order, not sorted like a map."""


def _shortest_f32(x: float) -> str:
    # shortest decimal string that round-trips through float32
    f = struct.unpack("f", struct.pack("f", x))[0]
    for prec in range(1, 18):
        s = f"{f:.{prec}g}"
        if struct.unpack("f", struct.pack("f", float(s)))[0] == f:
            return s
    return repr(f)


def _fmt_float(x: float, bits: int) -> str:
    if math.isnan(x) or math.isinf(x):
        raise ValueError(f"json: unsupported value: {x}")
    if x == 0:
        return "-0" if math.copysign(1.0, x) < 0 else "0"
    a = abs(x)
    if 1e-6 <= a < 1e21:  # Go's 'f' form: numpy's shortest round-trip digits, positional (fast path)
        v = _np.float32(x) if bits == 32 else _np.float64(x)
        if 1e-6 <= abs(float(v)) < 1e21:
            return _np.format_float_positional(v, unique=True, trim="-")
    return _fmt_float_slow(x, bits)


def _fmt_float_slow(x: float, bits: int) -> str:
    if x == 0:
        return "-0" if math.copysign(1.0, x) < 0 else "0"
    s = _shortest_f32(x) if bits == 32 else repr(float(x))
    from decimal import Decimal
    d = Decimal(s)
    a = abs(float(s))
    if a < 1e-6 or a >= 1e21:
        t = d.as_tuple()
        digits = "".join(map(str, t.digits)).rstrip("0") or "0"
        exp = len(t.digits) + t.exponent - 1
        m = digits[0] + ("." + digits[1:] if len(digits) > 1 else "")
        sign = "-" if t.sign else ""
        es = f"e-{abs(exp)}" if exp < 0 else f"e+{exp:02d}"  # Go cleans e-07 -> e-7
        return f"{sign}{m}{es}"
    out = format(d, "f")
    if "." in out:
        out = out.rstrip("0").rstrip(".")
    return out


_ESC = {'"': '\\"', "\\": "\\\\", "\n": "\\n", "\r": "\\r", "\t": "\\t", "<": "\\u003c", ">": "\\u003e",
        "&": "\\u0026", "\u2028": "\\u2028", "\u2029": "\\u2029", "\b": "\\b", "\f": "\\f"}


_HTML = ("<", ">", "&", "\u2028", "\u2029")


def _str(s: str) -> str:
    """C-accelerated JSON string escaping plus Go's HTML-safe escapes; lone surrogates (invalid
    UTF-8 in Go: text/preprocess.py truncate_preview keeps one per byte) take the slow path, which
    writes the ``\\ufffd`` escape for each, like Go."""
    if _SURR.search(s):
        return _str_slow(s)
    out = _encode_basestring(s)
    if any(c in out for c in _HTML):
        out = (out.replace("<", "\\u003c").replace(">", "\\u003e").replace("&", "\\u0026")
               .replace("\u2028", "\\u2028").replace("\u2029", "\\u2029"))
    return out


def _str_slow(s: str) -> str:
    out = ['"']
    for ch in s:
        e = _ESC.get(ch)
        if e is not None:
            out.append(e)
        elif ord(ch) < 0x20:
            out.append(f"\\u{ord(ch):04x}")
        elif 0xD800 <= ord(ch) <= 0xDFFF:
            out.append("\\ufffd")  # encoding/json: the escape, once per invalid byte
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


def _enc(v, ind: str, depth: int) -> str:
    if v is None:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, F32):
        return _fmt_float(float(v), 32)
    if isinstance(v, float):
        return _fmt_float(v, 64)
    if isinstance(v, int):
        return str(v)
    if isinstance(v, str):
        return _str(v)
    pad = ind * (depth + 1)
    end = ind * depth
    if isinstance(v, dict):
        if not v:
            return "{}"
        keys = list(v) if isinstance(v, Struct) else sorted(v, key=lambda s: str(s).encode())
        items = [f"{pad}{_str(str(k))}: {_enc(v[k], ind, depth + 1)}" for k in keys]
        return "{\n" + ",\n".join(items) + "\n" + end + "}"
    if isinstance(v, (list, tuple)):
        if not v:
            return "[]"
        items = [f"{pad}{_enc(x, ind, depth + 1)}" for x in v]
        return "[\n" + ",\n".join(items) + "\n" + end + "]"
    if hasattr(v, "to_json"):
        return _enc(v.to_json(), ind, depth)
    raise TypeError(f"cannot encode {type(v)}")


def dumps(v, indent: str = "  ") -> str:
    """Encode like Go's Encoder with SetIndent("", indent), including the trailing newline."""
    return _enc(v, indent, 0) + "\n"


def dumps_compact(v) -> str:
    """json.Marshal: no indentation, sorted map keys, no trailing newline."""
    return _compact(v)


def _compact(v) -> str:
    if isinstance(v, dict):
        keys = list(v) if isinstance(v, Struct) else sorted(v, key=lambda s: str(s).encode())
        return "{" + ",".join(f"{_str(str(k))}:{_compact(v[k])}" for k in keys) + "}"
    if isinstance(v, (list, tuple)):
        return "[" + ",".join(_compact(x) for x in v) + "]"
    return _enc(v, "", 0)
