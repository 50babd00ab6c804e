"""multipart/form-data parser (python-multipart is not installed; FastAPI ``File()`` needs it).

Mirrors what the gateway needs from Go's ``r.FormFile("file")`` (cmd/gateway/main.go:58): the
first part named ``file`` that carries a filename, with its part headers (Content-Type) and size.
"""
from __future__ import annotations

from dataclasses import dataclass, field


class MultipartError(ValueError):
    pass


@dataclass
class Part:
    name: str
    filename: str | None
    headers: dict = field(default_factory=dict)
    data: bytes = b""

    @property
    def content_type(self) -> str:
        return self.headers.get("content-type", "")

    @property
    def size(self) -> int:
        return len(self.data)


def _params(value: str) -> tuple[str, dict]:
    parts = [p.strip() for p in _split_semicolons(value)]
    main = parts[0].lower() if parts else ""
    params = {}
    for p in parts[1:]:
        if "=" not in p:
            continue
        k, v = p.split("=", 1)
        k = k.strip().lower()
        v = v.strip()
        if k.endswith("*") and "''" in v:  # RFC 5987 filename*=utf-8''...
            from urllib.parse import unquote
            k = k[:-1]
            v = unquote(v.split("''", 1)[1])
        elif len(v) >= 2 and v[0] == '"' and v[-1] == '"':
            v = v[1:-1].replace('\\"', '"').replace("\\\\", "\\")
        params[k] = v
    return main, params


def _split_semicolons(s: str):
    out, cur, q = [], [], False
    for ch in s:
        if ch == '"':
            q = not q
        if ch == ";" and not q:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    out.append("".join(cur))
    return out


def boundary_of(content_type: str) -> str:
    main, params = _params(content_type or "")
    if main != "multipart/form-data" and not main.startswith("multipart/"):
        raise MultipartError("request Content-Type isn't multipart/form-data")
    b = params.get("boundary")
    if not b:
        raise MultipartError("no multipart boundary param in Content-Type")
    return b


def parse(body: bytes, content_type: str) -> list[Part]:
    b = boundary_of(content_type).encode("latin-1")
    delim = b"--" + b
    parts = []
    pos = body.find(delim)
    if pos < 0:
        raise MultipartError("multipart: NextPart: EOF")
    pos += len(delim)
    while True:
        if body[pos:pos + 2] == b"--":
            break
        if body[pos:pos + 2] == b"\r\n":
            pos += 2
        elif body[pos:pos + 1] == b"\n":
            pos += 1
        hdr_end = body.find(b"\r\n\r\n", pos)
        sep = 4
        if hdr_end < 0:
            hdr_end = body.find(b"\n\n", pos)
            sep = 2
            if hdr_end < 0:
                raise MultipartError("multipart: malformed part headers")
        headers = {}
        for line in body[pos:hdr_end].split(b"\n"):
            line = line.rstrip(b"\r")
            if not line or b":" not in line:
                continue
            k, v = line.split(b":", 1)
            headers[k.decode("latin-1").strip().lower()] = v.decode("utf-8", "replace").strip()
        data_start = hdr_end + sep
        nxt = body.find(b"\r\n" + delim, data_start)
        strip = 2
        if nxt < 0:
            nxt = body.find(b"\n" + delim, data_start)
            strip = 1
            if nxt < 0:
                raise MultipartError("multipart: NextPart: EOF")
        data = body[data_start:nxt]
        _, cd = _params(headers.get("content-disposition", ""))
        parts.append(Part(cd.get("name", ""), cd.get("filename"), headers, data))
        pos = nxt + strip + len(delim)
        if pos >= len(body):
            break
    return parts


def form_file(body: bytes, content_type: str, field_name: str = "file") -> Part:
    """Go ``Request.FormFile``: first part with this field name and a filename."""
    for p in parse(body, content_type):
        if p.name == field_name and p.filename is not None:
            return p
    raise MultipartError("http: no such file")


def build(fields: dict, files: dict, boundary: str = "XdaBoundary7MA4YWxkTrZu0gW") -> tuple[bytes, str]:
    """Encode a multipart body (tests / clients). files: name -> (filename, data, content_type|None)."""
    out = []
    for k, v in fields.items():
        out.append(f'--{boundary}\r\nContent-Disposition: form-data; name="{k}"\r\n\r\n{v}\r\n'.encode())
    for k, (fn, data, ct) in files.items():
        h = f'--{boundary}\r\nContent-Disposition: form-data; name="{k}"; filename="{fn}"\r\n'
        if ct:
            h += f"Content-Type: {ct}\r\n"
        out.append(h.encode() + b"\r\n" + data + b"\r\n")
    out.append(f"--{boundary}--\r\n".encode())
    return b"".join(out), f"multipart/form-data; boundary={boundary}"
