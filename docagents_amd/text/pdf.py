"""Minimal PDF text extraction (no PDF library is available offline).

Replaces ledongthuc/pdf as used by the gateway (cmd/gateway/main.go:210-249): pages in page-tree
order, pages that are null or have no /Contents are skipped, a page whose content fails to decode
is skipped, and every extracted page is followed by "\\n". Any structural parse error raises
``PDFError`` so the caller can fall back to the raw bytes (main.go:212-217).

Supported: classic xref-less scanning of ``N G obj ... endobj`` (works for incremental updates
and broken xref tables), object streams (/ObjStm), FlateDecode / ASCIIHexDecode / ASCII85Decode
content streams, Tj / TJ / ' / " text operators, T* / Td / TD / Tm line breaks, simple fonts
(WinAnsi/latin-1 bytes) and /ToUnicode CMaps (bfchar / bfrange) for composite fonts.
"""
from __future__ import annotations

import re
import zlib


_LIT_SPECIAL = re.compile(rb"[\\()]")

class PDFError(ValueError):
    pass


class Ref:
    __slots__ = ("num", "gen")

    def __init__(self, num, gen):
        self.num, self.gen = num, gen

    def __repr__(self):
        return f"{self.num} {self.gen} R"


class Name(str):
    pass


class Stream:
    def __init__(self, d, raw):
        self.dict, self.raw = d, raw


_WS = b" \t\r\n\x0c\x00"
_DELIM = b"()<>[]{}/%"


class Lexer:
    def __init__(self, data: bytes, pos: int = 0):
        self.d, self.p = data, pos

    def skip(self):
        d, n = self.d, len(self.d)
        while self.p < n:
            c = d[self.p]
            if c in _WS:
                self.p += 1
            elif c == 0x25:  # %
                while self.p < n and d[self.p] not in b"\r\n":
                    self.p += 1
            else:
                break

    def token(self):
        self.skip()
        d, n = self.d, len(self.d)
        if self.p >= n:
            return None
        c = d[self.p]
        if c == 0x2F:  # /Name
            s = self.p + 1
            self.p = s
            while self.p < n and d[self.p] not in _WS and d[self.p] not in _DELIM:
                self.p += 1
            raw = d[s:self.p]
            return Name(re.sub(rb"#([0-9A-Fa-f]{2})", lambda m: bytes([int(m.group(1), 16)]), raw).decode("latin-1"))
        if c == 0x28:  # (string)
            return self._lit()
        if c == 0x3C:  # < hex or <<
            if self.p + 1 < n and d[self.p + 1] == 0x3C:
                self.p += 2
                return "<<"
            e = d.find(b">", self.p)
            if e < 0:
                raise PDFError("unterminated hex string")
            h = re.sub(rb"\s", b"", d[self.p + 1:e])
            self.p = e + 1
            if len(h) % 2:
                h += b"0"
            return bytes.fromhex(h.decode("latin-1")) if h else b""
        if c == 0x3E and self.p + 1 < n and d[self.p + 1] == 0x3E:
            self.p += 2
            return ">>"
        if c in b"[]{}":
            self.p += 1
            return chr(c)
        s = self.p
        while self.p < n and d[self.p] not in _WS and d[self.p] not in _DELIM:
            self.p += 1
        if self.p == s:
            self.p += 1
            return chr(c)
        w = d[s:self.p]
        try:
            if b"." in w:
                return float(w)
            return int(w)
        except ValueError:
            return w.decode("latin-1")  # keyword / operator

    def _lit(self) -> bytes:
        d, n = self.d, len(self.d)
        self.p += 1
        out = bytearray()
        depth = 1
        while self.p < n:
            # copy the run up to the next byte that matters ('\\', '(' or ')') in one slice: a
            # content stream is mostly long literal strings, byte-at-a-time Python was 70 % of extraction
            m_ = _LIT_SPECIAL.search(d, self.p)
            if m_ is None:
                break
            if m_.start() > self.p:
                out += d[self.p:m_.start()]
                self.p = m_.start()
            c = d[self.p]
            if c == 0x5C:  # backslash
                self.p += 1
                if self.p >= n:
                    break
                e = d[self.p]
                m = {0x6E: 10, 0x72: 13, 0x74: 9, 0x62: 8, 0x66: 12, 0x28: 0x28, 0x29: 0x29, 0x5C: 0x5C}
                if e in m:
                    out.append(m[e])
                    self.p += 1
                elif 0x30 <= e <= 0x37:
                    j = self.p
                    while j < n and j < self.p + 3 and 0x30 <= d[j] <= 0x37:
                        j += 1
                    out.append(int(d[self.p:j], 8) & 0xFF)
                    self.p = j
                elif e in b"\r\n":
                    self.p += 1
                    if e == 0x0D and self.p < n and d[self.p] == 0x0A:
                        self.p += 1
                else:
                    out.append(e)
                    self.p += 1
                continue
            if c == 0x28:
                depth += 1
            elif c == 0x29:
                depth -= 1
                if depth == 0:
                    self.p += 1
                    return bytes(out)
            out.append(c)
            self.p += 1
        raise PDFError("unterminated string")

    def obj(self, tok=None):
        t = self.token() if tok is None else tok
        if t == "<<":
            dct = {}
            while True:
                k = self.token()
                if k == ">>" or k is None:
                    return dct
                if not isinstance(k, Name):
                    raise PDFError("dict key is not a name")
                dct[str(k)] = self.obj()
        if t == "[":
            arr = []
            while True:
                x = self.token()
                if x == "]" or x is None:
                    return arr
                arr.append(self.obj(x))
        if isinstance(t, int):
            save = self.p
            t2 = self.token()
            if isinstance(t2, int):
                t3 = self.token()
                if t3 == "R":
                    return Ref(t, t2)
            self.p = save
            return t
        if t in ("true", "false"):
            return t == "true"
        if t == "null":
            return None
        return t


_OBJ_RE = re.compile(rb"(\d+)\s+(\d+)\s+obj\b")


class PDFDocument:
    def __init__(self, data: bytes):
        if not data.lstrip()[:5].startswith(b"%PDF"):
            raise PDFError("not a PDF file")
        self.data = data
        self.objs: dict[int, object] = {}
        self._scan()
        self._expand_objstms()

    def _scan(self):
        d = self.data
        for m in _OBJ_RE.finditer(d):
            num = int(m.group(1))
            lx = Lexer(d, m.end())
            try:
                o = lx.obj()
                lx.skip()
                if d.startswith(b"stream", lx.p) and isinstance(o, dict):
                    p = lx.p + 6
                    if d[p:p + 2] == b"\r\n":
                        p += 2
                    elif d[p:p + 1] in (b"\n", b"\r"):
                        p += 1
                    ln = o.get("Length")
                    end = None
                    if isinstance(ln, int) and d[p + ln:p + ln + 30].lstrip().startswith(b"endstream"):
                        end = p + ln
                    if end is None:
                        end = d.find(b"endstream", p)
                        if end < 0:
                            continue
                        while end > p and d[end - 1] in b"\r\n":
                            end -= 1
                    o = Stream(o, d[p:end])
                self.objs[num] = o  # later definitions (incremental updates) win
            except PDFError:
                continue

    def _expand_objstms(self):
        for num, o in list(self.objs.items()):
            if isinstance(o, Stream) and o.dict.get("Type") == "ObjStm":
                try:
                    raw = self.decode(o)
                    n = int(o.dict.get("N", 0))
                    first = int(o.dict.get("First", 0))
                    lx = Lexer(raw)
                    hdr = [lx.token() for _ in range(2 * n)]
                    for i in range(n):
                        onum, off = hdr[2 * i], hdr[2 * i + 1]
                        if onum not in self.objs:
                            self.objs[onum] = Lexer(raw, first + off).obj()
                except Exception:  # noqa: BLE001
                    continue

    def resolve(self, o, depth=0):
        while isinstance(o, Ref):
            if depth > 32:
                raise PDFError("reference loop")
            o = self.objs.get(o.num)
            depth += 1
        return o

    def decode(self, s: Stream) -> bytes:
        filt = self.resolve(s.dict.get("Filter"))
        filters = filt if isinstance(filt, list) else ([filt] if filt else [])
        data = s.raw
        for f in filters:
            f = self.resolve(f)
            if f in ("FlateDecode", "Fl"):
                try:
                    data = zlib.decompress(data)
                except zlib.error:
                    data = zlib.decompressobj().decompress(data)
            elif f in ("ASCIIHexDecode", "AHx"):
                h = re.sub(rb"\s", b"", data).rstrip(b">")
                data = bytes.fromhex(h.decode() + ("0" if len(h) % 2 else ""))
            elif f in ("ASCII85Decode", "A85"):
                import base64
                t = re.sub(rb"\s", b"", data)
                if t.startswith(b"<~"):
                    t = t[2:]
                data = base64.a85decode(t.rstrip(b"~>") + b"~>", adobe=True)
            else:
                raise PDFError(f"unsupported filter {f}")
        return data

    def pages(self) -> list:
        root = None
        for o in self.objs.values():
            if isinstance(o, Stream) and o.dict.get("Type") == "XRef" and "Root" in o.dict:
                root = o.dict["Root"]
        tm = self.data.rfind(b"trailer")
        if tm >= 0:
            try:
                t = Lexer(self.data, tm + 7).obj()
                if isinstance(t, dict) and "Root" in t:
                    root = t["Root"]
            except PDFError:
                pass
        cat = self.resolve(root)
        if not isinstance(cat, dict):
            for o in self.objs.values():
                if isinstance(o, dict) and o.get("Type") == "Catalog":
                    cat = o
                    break
        if not isinstance(cat, dict):
            raise PDFError("no document catalog")
        out = []
        self._walk(self.resolve(cat.get("Pages")), out, 0, {})
        return out

    def _walk(self, node, out, depth, inherited):
        if not isinstance(node, dict) or depth > 64:
            return
        inh = dict(inherited)
        if "Resources" in node:
            inh["Resources"] = node["Resources"]
        if node.get("Type") == "Pages" or "Kids" in node:
            for k in self.resolve(node.get("Kids")) or []:
                self._walk(self.resolve(k), out, depth + 1, inh)
        else:
            page = dict(node)
            page.setdefault("Resources", inh.get("Resources"))
            out.append(page)

    # ------------------------------------------------------------------ text
    def _fonts(self, page) -> dict:
        res = self.resolve(page.get("Resources")) or {}
        fonts = self.resolve(res.get("Font")) if isinstance(res, dict) else None
        out = {}
        for name, ref in (fonts or {}).items():
            f = self.resolve(ref)
            cmap = None
            if isinstance(f, dict) and "ToUnicode" in f:
                tu = self.resolve(f["ToUnicode"])
                if isinstance(tu, Stream):
                    try:
                        cmap = parse_tounicode(self.decode(tu))
                    except Exception:  # noqa: BLE001
                        cmap = None
            two = isinstance(f, dict) and f.get("Subtype") == "Type0"
            out[name] = (cmap, two)
        return out

    def page_text(self, page) -> str:
        contents = self.resolve(page.get("Contents"))
        streams = contents if isinstance(contents, list) else [contents]
        data = b""
        for s in streams:
            s = self.resolve(s)
            if isinstance(s, Stream):
                data += self.decode(s) + b"\n"
        return content_text(data, self._fonts(page))


def parse_tounicode(data: bytes) -> dict:
    m = {}
    for blk in re.findall(rb"beginbfchar(.*?)endbfchar", data, re.S):
        for a, b in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]+)>", blk):
            m[int(a, 16)] = bytes.fromhex(b.decode()).decode("utf-16-be", "replace")
    for blk in re.findall(rb"beginbfrange(.*?)endbfrange", data, re.S):
        for a, b, c in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]+)>\s*(<[0-9A-Fa-f]+>|\[[^\]]*\])", blk):
            lo, hi = int(a, 16), int(b, 16)
            if c.startswith(b"["):
                for i, h in enumerate(re.findall(rb"<([0-9A-Fa-f]+)>", c)):
                    m[lo + i] = bytes.fromhex(h.decode()).decode("utf-16-be", "replace")
            else:
                base = int(c[1:-1], 16)
                for i in range(hi - lo + 1):
                    try:
                        m[lo + i] = chr(base + i)
                    except ValueError:
                        pass
    return m


def _decode_str(s: bytes, font) -> str:
    cmap, two = font if font else (None, False)
    if cmap:
        if two:
            return "".join(cmap.get((s[i] << 8) | s[i + 1], "") for i in range(0, len(s) - 1, 2))
        return "".join(cmap.get(b, chr(b)) for b in s)
    if two:
        return s.decode("utf-16-be", "replace")
    return s.decode("latin-1")


def content_text(data: bytes, fonts: dict) -> str:
    lx = Lexer(data)
    out: list[str] = []
    stack: list = []
    font = None
    while True:
        t = lx.token()
        if t is None:
            break
        if t in ("[", "<<"):
            stack.append(lx.obj(t))
            continue
        if isinstance(t, str) and not isinstance(t, Name) and t not in ("]", ">>") and not isinstance(t, bytes):
            op = t
            if op == "Tf" and len(stack) >= 2:
                font = fonts.get(str(stack[-2]))
            elif op == "Tj" and stack and isinstance(stack[-1], bytes):
                out.append(_decode_str(stack[-1], font))
            elif op == "TJ" and stack and isinstance(stack[-1], list):
                for x in stack[-1]:
                    if isinstance(x, bytes):
                        out.append(_decode_str(x, font))
                    elif isinstance(x, (int, float)) and x < -200:
                        out.append(" ")
            elif op in ("'", '"') and stack and isinstance(stack[-1], bytes):
                out.append("\n")
                out.append(_decode_str(stack[-1], font))
            elif op == "T*":
                out.append("\n")
            elif op in ("Td", "TD") and len(stack) >= 2 and isinstance(stack[-1], (int, float)) and stack[-1] != 0:
                out.append("\n")
            elif op == "Tm" and out and out[-1] != "\n":
                out.append("\n")
            elif op == "BI":  # inline image: skip to EI
                e = data.find(b"EI", lx.p)
                lx.p = len(data) if e < 0 else e + 2
            stack.clear()
            continue
        stack.append(t)
    text = "".join(out)
    return re.sub(r"\n{2,}", "\n", text).strip("\n")


def extract_text(data: bytes) -> str:
    """GetPlainText per page + "\\n" (cmd/gateway/main.go:223-249)."""
    doc = PDFDocument(data)
    parts = []
    for page in doc.pages():
        if page is None or page.get("Contents") is None:
            continue
        try:
            txt = doc.page_text(page)
        except Exception:  # noqa: BLE001 - skip pages that fail to extract
            continue
        parts.append(txt)
        parts.append("\n")
    return "".join(parts)


def make_pdf(pages: list[str], compress: bool = True) -> bytes:
    """Write a small valid PDF (Helvetica, one text line per input line) — tests and benchmarks."""
    objs = []

    def add(b: bytes) -> int:
        objs.append(b)
        return len(objs)

    font = add(b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica /Encoding /WinAnsiEncoding >>")
    page_ids = []
    pages_id_placeholder = len(objs) + 1 + 2 * len(pages)
    for text in pages:
        lines = text.split("\n")
        ops = [b"BT", b"/F1 11 Tf", b"14 TL", b"50 780 Td"]
        for i, ln in enumerate(lines):
            esc = ln.encode("latin-1", "replace").replace(b"\\", b"\\\\").replace(b"(", b"\\(").replace(b")", b"\\)")
            ops.append(b"(" + esc + b") Tj" + (b" T*" if i < len(lines) - 1 else b""))
        ops.append(b"ET")
        raw = b"\n".join(ops)
        if compress:
            body = zlib.compress(raw)
            cs = add(b"<< /Length %d /Filter /FlateDecode >>\nstream\n" % len(body) + body + b"\nendstream")
        else:
            cs = add(b"<< /Length %d >>\nstream\n" % len(raw) + raw + b"\nendstream")
        page_ids.append(add(b"<< /Type /Page /Parent %d 0 R /MediaBox [0 0 612 792] /Contents %d 0 R "
                            b"/Resources << /Font << /F1 %d 0 R >> >> >>" % (pages_id_placeholder, cs, font)))
    kids = b" ".join(b"%d 0 R" % p for p in page_ids)
    pages_id = add(b"<< /Type /Pages /Kids [" + kids + b"] /Count %d >>" % len(page_ids))
    assert pages_id == pages_id_placeholder
    cat = add(b"<< /Type /Catalog /Pages %d 0 R >>" % pages_id)
    out = bytearray(b"%PDF-1.4\n%\xe2\xe3\xcf\xd3\n")
    offs = []
    for i, o in enumerate(objs, 1):
        offs.append(len(out))
        out += b"%d 0 obj\n" % i + o + b"\nendobj\n"
    xref = len(out)
    out += b"xref\n0 %d\n0000000000 65535 f \n" % (len(objs) + 1)
    for off in offs:
        out += b"%010d 00000 n \n" % off
    out += b"trailer\n<< /Size %d /Root %d 0 R >>\nstartxref\n%d\n%%%%EOF\n" % (len(objs) + 1, cat, xref)
    return bytes(out)
