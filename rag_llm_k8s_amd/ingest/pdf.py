"""Self-contained PDF text extractor (replaces PyPDF2.PdfReader.extract_text, D7).

Reference behaviour (/root/reference/llm/rag.py:47-52): for every page, append
``page.extract_text() + "\\n"``; the result is whitespace-split into words by the
chunker, so what matters for parity is the *word sequence*, not exact layout.

Supported: classic xref tables and PDF 1.5 cross-reference / object streams (objects
are located by scanning, then /ObjStm containers are expanded), FlateDecode /
ASCIIHexDecode / ASCII85Decode stream filters, page-tree inheritance of /Resources,
simple fonts with Standard/WinAnsi/MacRoman encodings and /Differences, Type0 fonts
through /ToUnicode CMaps (bfchar / bfrange), Form XObjects (``Do``) and the text
operators BT/ET Tf Tj TJ ' " Td TD Tm T* TL. Line breaks are emitted on vertical text
moves, spaces on large negative TJ adjustments (word gaps), like PyPDF2's non-layout mode.
"""
from __future__ import annotations

import io
import re
import zlib

WS = b" \t\r\n\f\x00"
DELIM = b"()<>[]{}/%"


class Ref:
    __slots__ = ("num", "gen")

    def __init__(self, num, gen):
        self.num, self.gen = num, gen

    def __repr__(self):
        return "Ref(%d,%d)" % (self.num, self.gen)


class Name(str):
    pass


class Stream:
    def __init__(self, d, raw):
        self.dict, self.raw = d, raw


class Op(str):
    pass


class _Lexer:
    def __init__(self, data: bytes, pos: int = 0):
        self.d, self.p, self.n = data, pos, len(data)

    def skip_ws(self):
        d, n = self.d, self.n
        while self.p < n:
            c = d[self.p]
            if c in WS:
                self.p += 1
            elif c == 0x25:  # %
                while self.p < n and d[self.p] not in b"\r\n":
                    self.p += 1
            else:
                break

    def token(self):
        """Next raw token: bytes for structural tokens/keywords/numbers, or a parsed
        string (bytes wrapped in tuple ('str', b)), or ('name', str)."""
        self.skip_ws()
        d = self.d
        if self.p >= self.n:
            return None
        c = d[self.p]
        if c == 0x28:  # (
            return ("str", self._lit_string())
        if c == 0x3C:  # <
            if self.p + 1 < self.n and d[self.p + 1] == 0x3C:
                self.p += 2
                return b"<<"
            return ("str", self._hex_string())
        if c == 0x3E:
            if self.p + 1 < self.n and d[self.p + 1] == 0x3E:
                self.p += 2
                return b">>"
            self.p += 1
            return b">"
        if c in b"[]{}":
            self.p += 1
            return bytes([c])
        if c == 0x2F:  # /
            self.p += 1
            s = self.p
            while self.p < self.n and d[self.p] not in WS and d[self.p] not in DELIM:
                self.p += 1
            raw = d[s:self.p]
            raw = re.sub(rb"#([0-9A-Fa-f]{2})", lambda m: bytes([int(m.group(1), 16)]), raw)
            return ("name", raw.decode("latin-1"))
        s = self.p
        while self.p < self.n and d[self.p] not in WS and d[self.p] not in DELIM:
            self.p += 1
        if self.p == s:  # stray delimiter
            self.p += 1
        return d[s:self.p]

    def _lit_string(self):
        d = self.d
        self.p += 1
        out = bytearray()
        depth = 1
        while self.p < self.n:
            c = d[self.p]
            self.p += 1
            if c == 0x5C:  # backslash
                if self.p >= self.n:
                    break
                e = d[self.p]
                self.p += 1
                m = {0x6E: 10, 0x72: 13, 0x74: 9, 0x62: 8, 0x66: 12, 0x28: 0x28, 0x29: 0x29, 0x5C: 0x5C}
                if e in m:
                    out.append(m[e])
                elif 0x30 <= e <= 0x37:
                    v = e - 0x30
                    for _ in range(2):
                        if self.p < self.n and 0x30 <= d[self.p] <= 0x37:
                            v = v * 8 + d[self.p] - 0x30
                            self.p += 1
                    out.append(v & 0xFF)
                elif e == 0x0D:
                    if self.p < self.n and d[self.p] == 0x0A:
                        self.p += 1
                elif e == 0x0A:
                    pass
                else:
                    out.append(e)
            elif c == 0x28:
                depth += 1
                out.append(c)
            elif c == 0x29:
                depth -= 1
                if depth == 0:
                    break
                out.append(c)
            else:
                out.append(c)
        return bytes(out)

    def _hex_string(self):
        d = self.d
        self.p += 1
        e = d.find(b">", self.p)
        if e < 0:
            e = self.n
        h = re.sub(rb"[^0-9A-Fa-f]", b"", d[self.p:e])
        self.p = e + 1
        if len(h) % 2:
            h += b"0"
        return bytes.fromhex(h.decode("ascii"))


def _num(tok):
    try:
        if b"." in tok:
            return float(tok)
        return int(tok)
    except ValueError:
        return None


def parse_object(lex: _Lexer):
    """Parse one PDF object (no stream handling)."""
    t = lex.token()
    return _obj_from(lex, t)


def _obj_from(lex, t):
    if t is None:
        return None
    if isinstance(t, tuple):
        return Name(t[1]) if t[0] == "name" else t[1]
    if t == b"<<":
        d = {}
        while True:
            k = lex.token()
            if k is None or k == b">>":
                return d
            if isinstance(k, tuple) and k[0] == "name":
                d[k[1]] = parse_object(lex)
    if t == b"[":
        arr = []
        while True:
            save = lex.p
            k = lex.token()
            if k is None or k == b"]":
                return arr
            v = _obj_from(lex, k)
            # n g R inside arrays
            if isinstance(v, int) and not isinstance(v, bool):
                save2 = lex.p
                t2 = lex.token()
                if isinstance(t2, bytes) and _num(t2) is not None and isinstance(_num(t2), int):
                    t3 = lex.token()
                    if t3 == b"R":
                        arr.append(Ref(v, _num(t2)))
                        continue
                lex.p = save2
            arr.append(v)
            del save
    if t in (b"true", b"false"):
        return t == b"true"
    if t == b"null":
        return None
    n = _num(t)
    if n is not None:
        if isinstance(n, int):
            save = lex.p
            t2 = lex.token()
            if isinstance(t2, bytes) and isinstance(_num(t2), int):
                t3 = lex.token()
                if t3 == b"R":
                    return Ref(n, _num(t2))
            lex.p = save
        return n
    return Op(t.decode("latin-1"))


# --------------------------------------------------------------------------- filters
def _ascii85(data):
    data = re.sub(rb"\s", b"", data)
    if data.startswith(b"<~"):
        data = data[2:]
    e = data.find(b"~>")
    if e >= 0:
        data = data[:e]
    out = bytearray()
    group = []
    for c in data:
        if c == ord("z") and not group:
            out += b"\0\0\0\0"
            continue
        group.append(c - 33)
        if len(group) == 5:
            v = 0
            for g in group:
                v = v * 85 + g
            out += v.to_bytes(4, "big")
            group = []
    if group:
        n = len(group)
        group += [84] * (5 - n)
        v = 0
        for g in group:
            v = v * 85 + g
        out += v.to_bytes(4, "big")[: n - 1]
    return bytes(out)


def _predictor(data, parms):
    if not parms:
        return data
    pred = parms.get("Predictor", 1)
    if pred < 10:
        return data
    cols = parms.get("Columns", 1) * parms.get("Colors", 1) * parms.get("BitsPerComponent", 8) // 8
    bpp = max(1, parms.get("Colors", 1) * parms.get("BitsPerComponent", 8) // 8)
    out = bytearray()
    prev = bytearray(cols)
    i = 0
    while i < len(data):
        ft = data[i]
        row = bytearray(data[i + 1:i + 1 + cols])
        i += 1 + cols
        for j in range(len(row)):
            a = row[j - bpp] if j >= bpp else 0
            b = prev[j] if j < len(prev) else 0
            c = prev[j - bpp] if j >= bpp else 0
            if ft == 1:
                row[j] = (row[j] + a) & 255
            elif ft == 2:
                row[j] = (row[j] + b) & 255
            elif ft == 3:
                row[j] = (row[j] + (a + b) // 2) & 255
            elif ft == 4:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                row[j] = (row[j] + (a if pa <= pb and pa <= pc else (b if pb <= pc else c))) & 255
        out += row
        prev = row
    return bytes(out)


def decode_stream(doc, s: Stream) -> bytes:
    f = doc.resolve(s.dict.get("Filter"))
    parms = doc.resolve(s.dict.get("DecodeParms"))
    filters = f if isinstance(f, list) else ([f] if f else [])
    parms = parms if isinstance(parms, list) else [parms] * len(filters)
    data = s.raw
    for flt, pm in zip(filters, parms):
        flt = doc.resolve(flt)
        pm = doc.resolve(pm)
        if flt in ("FlateDecode", "Fl"):
            try:
                data = zlib.decompress(data)
            except zlib.error:
                d = zlib.decompressobj()
                try:
                    data = d.decompress(data)
                except zlib.error:
                    return b""
            data = _predictor(data, pm if isinstance(pm, dict) else None)
        elif flt in ("ASCIIHexDecode", "AHx"):
            h = re.sub(rb"[^0-9A-Fa-f]", b"", data.split(b">")[0])
            data = bytes.fromhex((h + b"0" * (len(h) % 2)).decode())
        elif flt in ("ASCII85Decode", "A85"):
            data = _ascii85(data)
        else:  # images (DCT, JBIG2, ...) are irrelevant for text
            return b""
    return data


# --------------------------------------------------------------------------- document
_OBJ_RE = re.compile(rb"(\d+)\s+(\d+)\s+obj\b")


class PdfDocument:
    def __init__(self, data: bytes):
        self.data = data
        self.objects = {}
        self.trailer = {}
        self._scan()

    def _scan(self):
        d = self.data
        pos = 0
        while True:
            m = _OBJ_RE.search(d, pos)
            if not m:
                break
            num = int(m.group(1))
            lex = _Lexer(d, m.end())
            try:
                obj = parse_object(lex)
            except Exception:
                pos = m.end()
                continue
            save = lex.p
            t = lex.token()
            if t == b"stream" and isinstance(obj, dict):
                p = lex.p
                if d[p:p + 2] == b"\r\n":
                    p += 2
                elif d[p:p + 1] in (b"\n", b"\r"):
                    p += 1
                length = obj.get("Length")
                raw = None
                if isinstance(length, int) and d[p + length:p + length + 30].lstrip().startswith(b"endstream"):
                    raw = d[p:p + length]
                    end = p + length
                else:
                    e = d.find(b"endstream", p)
                    if e < 0:
                        e = len(d)
                    raw = d[p:e].rstrip(b"\r\n")
                    end = e
                obj = Stream(obj, raw)
                pos = end
            else:
                lex.p = save
                pos = lex.p
            self.objects[num] = obj
            if isinstance(obj, Stream) and obj.dict.get("Type") == "XRef":
                self.trailer.update({k: v for k, v in obj.dict.items() if k in ("Root", "Info")})
        for m in re.finditer(rb"trailer\s*<<", d):
            lex = _Lexer(d, m.end() - 2)
            try:
                t = parse_object(lex)
                if isinstance(t, dict):
                    self.trailer.update({k: v for k, v in t.items() if k in ("Root", "Info")})
            except Exception:
                pass
        # expand object streams
        for num, obj in list(self.objects.items()):
            if isinstance(obj, Stream) and obj.dict.get("Type") == "ObjStm":
                try:
                    self._expand_objstm(obj)
                except Exception:
                    continue

    def _expand_objstm(self, s):
        data = decode_stream(self, s)
        n = self.resolve(s.dict.get("N"))
        first = self.resolve(s.dict.get("First"))
        head = _Lexer(data, 0)
        pairs = []
        for _ in range(n):
            a = _num(head.token())
            b = _num(head.token())
            pairs.append((a, b))
        for onum, off in pairs:
            if onum in self.objects and not isinstance(self.objects[onum], Stream):
                pass
            lex = _Lexer(data, first + off)
            self.objects.setdefault(onum, parse_object(lex))

    def resolve(self, o, depth=0):
        while isinstance(o, Ref) and depth < 32:
            o = self.objects.get(o.num)
            depth += 1
        return o

    def catalog(self):
        root = self.resolve(self.trailer.get("Root"))
        if isinstance(root, dict):
            return root
        for o in self.objects.values():
            if isinstance(o, dict) and o.get("Type") == "Catalog":
                return o
        return {}

    def pages(self):
        out = []
        root = self.resolve(self.catalog().get("Pages"))

        def walk(node, inherited, seen):
            node = self.resolve(node)
            if not isinstance(node, dict) or id(node) in seen:
                return
            seen.add(id(node))
            inh = dict(inherited)
            for k in ("Resources", "MediaBox"):
                if k in node:
                    inh[k] = node[k]
            kids = self.resolve(node.get("Kids"))
            if node.get("Type") == "Pages" or isinstance(kids, list):
                for k in kids or []:
                    walk(k, inh, seen)
            else:
                page = dict(inh)
                page.update(node)
                out.append(page)

        if root is not None:
            walk(root, {}, set())
        if not out:  # no usable page tree: fall back to every /Page object
            out = [o for o in self.objects.values() if isinstance(o, dict) and o.get("Type") == "Page"]
        return out

    def page_content(self, page) -> bytes:
        c = self.resolve(page.get("Contents"))
        parts = c if isinstance(c, list) else [c]
        buf = []
        for p in parts:
            p = self.resolve(p)
            if isinstance(p, Stream):
                buf.append(decode_stream(self, p))
        return b"\n".join(buf)


# --------------------------------------------------------------------------- fonts
_MACROMAN_HI = ("ÄÅÇÉÑÖÜáàâäãåçéèêëíìîïñóòôöõúùûü†°¢£§•¶ß®©™´¨≠ÆØ∞±≤≥¥µ∂∑∏π∫ªºΩæø¿¡¬√ƒ≈∆«»… ÀÃÕŒœ–—“”‘’÷◊ÿŸ⁄€‹›ﬁﬂ‡·‚„‰ÂÊÁËÈÍÎÏÌÓÔ"
                "ÒÚÛÙıˆ˜¯˘˙˚¸˝˛ˇ")
_GLYPHS = {
    "space": " ", "quotesingle": "'", "quoteright": "’", "quoteleft": "‘", "quotedblleft": "“",
    "quotedblright": "”", "endash": "–", "emdash": "—", "bullet": "•", "fi": "fi", "fl": "fl",
    "ff": "ff", "ffi": "ffi", "ffl": "ffl", "ellipsis": "…", "hyphen": "-", "minus": "-", "period": ".",
    "comma": ",", "colon": ":", "semicolon": ";", "exclam": "!", "question": "?", "parenleft": "(",
    "parenright": ")", "bracketleft": "[", "bracketright": "]", "slash": "/", "ampersand": "&", "at": "@",
    "numbersign": "#", "dollar": "$", "percent": "%", "asterisk": "*", "plus": "+", "equal": "=", "less": "<",
    "greater": ">", "underscore": "_", "quotedbl": '"', "zero": "0", "one": "1", "two": "2", "three": "3",
    "four": "4", "five": "5", "six": "6", "seven": "7", "eight": "8", "nine": "9", "copyright": "©",
    "registered": "®", "trademark": "™", "degree": "°", "nbspace": " ",
}


def _glyph_to_unicode(name):
    if name in _GLYPHS:
        return _GLYPHS[name]
    if len(name) == 1:
        return name
    m = re.match(r"^uni([0-9A-Fa-f]{4})", name)
    if m:
        return chr(int(m.group(1), 16))
    m = re.match(r"^u([0-9A-Fa-f]{4,6})$", name)
    if m:
        return chr(int(m.group(1), 16))
    return ""


def _base_encoding(name):
    if name == "MacRomanEncoding":
        return [chr(i) if i < 128 else (_MACROMAN_HI[i - 128] if i - 128 < len(_MACROMAN_HI) else "")
                for i in range(256)]
    # WinAnsi (cp1252) also serves Standard encoding for printable ASCII
    out = []
    for i in range(256):
        try:
            out.append(bytes([i]).decode("cp1252"))
        except UnicodeDecodeError:
            out.append("")
    if name == "StandardEncoding":
        out[0x27] = "’"
        out[0x60] = "‘"
    return out


def parse_cmap(data: bytes):
    """ToUnicode CMap -> (code_bytes, {code: str})."""
    m = {}
    width = 1
    cs = re.search(rb"begincodespacerange(.*?)endcodespacerange", data, re.S)
    if cs:
        hx = re.findall(rb"<([0-9A-Fa-f]+)>", cs.group(1))
        if hx:
            width = max(1, len(hx[0]) // 2)

    def u(h):
        b = bytes.fromhex(h.decode())
        try:
            return b.decode("utf-16-be")
        except UnicodeDecodeError:
            return ""

    for blk in re.findall(rb"beginbfchar(.*?)endbfchar", data, re.S):
        for a, b in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]*)>", blk):
            m[int(a, 16)] = u(b)
            width = max(width, len(a) // 2) if len(a) // 2 <= 2 else width
    for blk in re.findall(rb"beginbfrange(.*?)endbfrange", data, re.S):
        for a, b, rest in re.findall(rb"<([0-9A-Fa-f]+)>\s*<([0-9A-Fa-f]+)>\s*(\[[^\]]*\]|<[0-9A-Fa-f]*>)", blk):
            lo, hi = int(a, 16), int(b, 16)
            if rest.startswith(b"["):
                vals = re.findall(rb"<([0-9A-Fa-f]*)>", rest)
                for i, v in enumerate(vals):
                    if lo + i <= hi:
                        m[lo + i] = u(v)
            else:
                base = bytes.fromhex(rest[1:-1].decode())
                if not base:
                    continue
                for i in range(min(hi - lo + 1, 65536)):
                    bb = bytearray(base)
                    bb[-1] = (bb[-1] + i) & 0xFF
                    try:
                        m[lo + i] = bytes(bb).decode("utf-16-be")
                    except UnicodeDecodeError:
                        m[lo + i] = ""
    return width, m


class Font:
    def __init__(self, doc, fdict):
        fdict = doc.resolve(fdict) or {}
        self.width = 1
        self.cmap = None
        self.enc = None
        sub = fdict.get("Subtype")
        tu = doc.resolve(fdict.get("ToUnicode"))
        if isinstance(tu, Stream):
            try:
                self.width, self.cmap = parse_cmap(decode_stream(doc, tu))
            except Exception:
                self.cmap = None
        if sub == "Type0":
            self.width = 2 if self.cmap is None else max(1, min(self.width, 4))
        else:
            self.width = 1  # simple fonts always use 1-byte codes, whatever the CMap codespace says
        if sub != "Type0":
            enc = doc.resolve(fdict.get("Encoding"))
            base = "StandardEncoding"
            diffs = None
            if isinstance(enc, str):
                base = enc
            elif isinstance(enc, dict):
                base = enc.get("BaseEncoding", "StandardEncoding")
                diffs = doc.resolve(enc.get("Differences"))
            table = _base_encoding(base)
            if diffs:
                code = 0
                for x in diffs:
                    x = doc.resolve(x)
                    if isinstance(x, int):
                        code = x
                    elif isinstance(x, str):
                        if 0 <= code < 256:
                            table[code] = _glyph_to_unicode(str(x))
                        code += 1
            self.enc = table

    def decode(self, b: bytes) -> str:
        if self.cmap is not None:
            out = []
            w = self.width
            i = 0
            while i + w <= len(b):
                code = int.from_bytes(b[i:i + w], "big")
                ch = self.cmap.get(code)
                if ch is None and self.enc is not None and code < 256:
                    ch = self.enc[code]
                out.append(ch or "")
                i += w
            return "".join(out)
        if self.width == 2:
            return ""  # CID font without ToUnicode: not decodable
        return "".join(self.enc[c] for c in b)


# --------------------------------------------------------------------------- content
def _content_ops(data: bytes):
    lex = _Lexer(data)
    operands = []
    while True:
        t = lex.token()
        if t is None:
            return
        if t == b"BI":  # inline image: skip to EI
            e = data.find(b"EI", lex.p)
            lex.p = len(data) if e < 0 else e + 2
            operands = []
            continue
        v = _obj_from(lex, t)
        if isinstance(v, Op):
            yield str(v), operands
            operands = []
        else:
            operands.append(v)


class _TextState:
    def __init__(self):
        self.out = []
        self.last_y = None
        self.tl = 0.0

    def emit(self, s):
        if s:
            self.out.append(s)

    def newline(self):
        if self.out and not self.out[-1].endswith("\n"):
            self.out.append("\n")


def _extract(doc, content, resources, st, depth=0):
    resources = doc.resolve(resources) or {}
    fonts = doc.resolve(resources.get("Font")) or {}
    xobjs = doc.resolve(resources.get("XObject")) or {}
    font_cache = {}
    cur = None
    ty_line = 0.0
    for op, args in _content_ops(content):
        if op == "Tf" and args:
            name = args[0]
            if name not in font_cache:
                font_cache[name] = Font(doc, fonts.get(name)) if isinstance(fonts, dict) else None
            cur = font_cache[name]
        elif op in ("Tj", "'", '"'):
            if op in ("'", '"'):
                st.newline()
            s = args[-1] if args else b""
            if isinstance(s, bytes) and cur is not None:
                st.emit(cur.decode(s))
        elif op == "TJ":
            arr = args[0] if args and isinstance(args[0], list) else []
            for x in arr:
                if isinstance(x, bytes):
                    if cur is not None:
                        st.emit(cur.decode(x))
                elif isinstance(x, (int, float)) and x < -250:
                    if st.out and not st.out[-1].endswith((" ", "\n")):
                        st.emit(" ")
        elif op in ("Td", "TD"):
            if len(args) >= 2 and isinstance(args[1], (int, float)):
                if abs(args[1]) > 1e-6:
                    st.newline()
                    ty_line = args[1]
                elif isinstance(args[0], (int, float)) and args[0] > 1e-6:
                    if st.out and not st.out[-1].endswith((" ", "\n")):
                        st.emit(" ")
                if op == "TD":
                    st.tl = -args[1]
        elif op == "Tm":
            if len(args) >= 6 and isinstance(args[5], (int, float)):
                y = args[5]
                if st.last_y is None or abs(y - st.last_y) > 1e-6:
                    if st.last_y is not None:
                        st.newline()
                st.last_y = y
        elif op == "T*":
            st.newline()
        elif op == "TL" and args:
            st.tl = args[0] if isinstance(args[0], (int, float)) else st.tl
        elif op == "ET":
            pass
        elif op == "Do" and args and depth < 8:
            xo = doc.resolve(xobjs.get(args[0])) if isinstance(xobjs, dict) else None
            if isinstance(xo, Stream) and xo.dict.get("Subtype") == "Form":
                _extract(doc, decode_stream(doc, xo), xo.dict.get("Resources", resources), st, depth + 1)
    del ty_line


def extract_pages(data: bytes):
    doc = PdfDocument(data)
    texts = []
    for page in doc.pages():
        st = _TextState()
        try:
            _extract(doc, doc.page_content(page), page.get("Resources"), st)
        except Exception:
            pass
        texts.append("".join(st.out))
    return texts


def extract_text(src) -> str:
    """Reference process_pdf text assembly: ''.join(page_text + '\\n')."""
    if hasattr(src, "read"):
        data = src.read()
    elif isinstance(src, (bytes, bytearray)):
        data = bytes(src)
    else:
        with open(src, "rb") as f:
            data = f.read()
    return "".join(t + "\n" for t in extract_pages(data))


# --------------------------------------------------------------------------- writer
def _pdf_escape(s: str) -> bytes:
    b = s.encode("cp1252", errors="replace")
    return b.replace(b"\\", b"\\\\").replace(b"(", b"\\(").replace(b")", b"\\)")


def write_pdf(pages, compress=True, object_streams=False, line_height=14, font_size=11) -> bytes:
    """Minimal PDF writer for synthetic corpora. `pages` is a list of lists of text
    lines (Helvetica, WinAnsiEncoding). With object_streams=True, non-stream objects
    go into an /ObjStm and a cross-reference stream replaces the xref table."""
    objs = {}
    font_id, pages_id, cat_id = 3, 2, 1
    next_id = 4
    page_ids = []
    contents = {}
    for lines in pages:
        cid, pid = next_id, next_id + 1
        next_id += 2
        y = 800
        ops = [b"BT", b"/F1 %d Tf" % font_size, b"%d TL" % line_height, b"50 %d Td" % y]
        for i, ln in enumerate(lines):
            if i:
                ops.append(b"T*")
            ops.append(b"(" + _pdf_escape(ln) + b") Tj")
        ops.append(b"ET")
        raw = b"\n".join(ops)
        contents[cid] = raw
        objs[pid] = b"<< /Type /Page /Parent 2 0 R /MediaBox [0 0 612 842] /Contents %d 0 R >>" % cid
        page_ids.append(pid)
    objs[cat_id] = b"<< /Type /Catalog /Pages 2 0 R >>"
    kids = b" ".join(b"%d 0 R" % p for p in page_ids)
    objs[pages_id] = (b"<< /Type /Pages /Kids [" + kids + b"] /Count %d /Resources << /Font << /F1 3 0 R >> >> >>"
                      % len(page_ids))
    objs[font_id] = b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica /Encoding /WinAnsiEncoding >>"

    out = io.BytesIO()
    out.write(b"%PDF-1.7\n%\xe2\xe3\xcf\xd3\n")
    offsets = {}

    def stream_obj(num, d, data):
        offsets[num] = out.tell()
        out.write(b"%d 0 obj\n" % num + d + b"\nstream\n" + data + b"\nendstream\nendobj\n")

    for cid, raw in contents.items():
        if compress:
            data = zlib.compress(raw)
            stream_obj(cid, b"<< /Length %d /Filter /FlateDecode >>" % len(data), data)
        else:
            stream_obj(cid, b"<< /Length %d >>" % len(raw), raw)
    if object_streams:
        nums = sorted(objs)
        body, header = b"", []
        for n in nums:
            header.append(b"%d %d" % (n, len(body)))
            body += objs[n] + b"\n"
        head = b" ".join(header) + b"\n"
        data = zlib.compress(head + body)
        osid = next_id
        stream_obj(osid, b"<< /Type /ObjStm /N %d /First %d /Length %d /Filter /FlateDecode >>"
                   % (len(nums), len(head), len(data)), data)
        xid = osid + 1
        xref_pos = out.tell()
        size = xid + 1
        rows = bytearray()
        for i in range(size):
            if i in offsets:
                rows += bytes([1]) + offsets[i].to_bytes(4, "big") + b"\0"
            elif i in objs:
                rows += bytes([2]) + osid.to_bytes(4, "big") + bytes([nums.index(i)])
            elif i == xid:
                rows += bytes([1]) + xref_pos.to_bytes(4, "big") + b"\0"
            else:
                rows += bytes([0, 0, 0, 0, 0, 255])
        xd = zlib.compress(bytes(rows))
        out.write(b"%d 0 obj\n<< /Type /XRef /Size %d /W [1 4 1] /Root 1 0 R /Length %d /Filter /FlateDecode >>"
                  b"\nstream\n" % (xid, size, len(xd)) + xd + b"\nendstream\nendobj\n")
        out.write(b"startxref\n%d\n%%%%EOF\n" % xref_pos)
        return out.getvalue()
    for n in sorted(objs):
        offsets[n] = out.tell()
        out.write(b"%d 0 obj\n" % n + objs[n] + b"\nendobj\n")
    xref_pos = out.tell()
    size = max(offsets) + 1
    out.write(b"xref\n0 %d\n0000000000 65535 f \n" % size)
    for i in range(1, size):
        out.write(b"%010d 00000 n \n" % offsets[i] if i in offsets else b"0000000000 65535 f \n")
    out.write(b"trailer\n<< /Size %d /Root 1 0 R >>\nstartxref\n%d\n%%%%EOF\n" % (size, xref_pos))
    return out.getvalue()
