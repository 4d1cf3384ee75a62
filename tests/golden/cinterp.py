"""cinterp -- a small interpreter for the C subset of the reference's DSP code.

TEST INFRASTRUCTURE ONLY (dev container): tests/golden/gen_fixtures.py uses it
to EXECUTE THE REFERENCE'S OWN FUNCTION BODIES (av1_fwd_txfm2d_*_c,
quantize_fp_helper_c, aom_quantize_b_helper_c, inv_txfm2d_add_c, sad(),
variance(), av1_build_quantizer, ...) read as text from /root/reference, and
turns their outputs into committed golden fixtures (tests/golden/*.npz).  The
reference cannot be compiled here under the round rules (its sources need
CMake-generated config/*.h headers); interpreting the text needs
no generated file: preprocessor conditionals take the defaults of
build/cmake/aom_config_defaults.cmake (parsed from the reference too), and an
undefined `foo` call resolves to `foo_c`, exactly what rtcd.pl's single-
implementation mode emits (`#define foo foo_c`, build/cmake/rtcd.pl:144-166).
Nothing here is imported by the product, by bench.py or by any -m gpu test.

C semantics kept exactly (LP64, gcc on x86-64, which is what the reference's
tests run under):
* integer types wrap to their width on every store and every arithmetic
  result (two's complement; signed overflow wraps as gcc's generated code
  does -- half_btf's int32 products rely on it, av1/common/av1_txfm.h:80);
* integer promotions and the usual arithmetic conversions (C11 6.3.1);
* `/` and `%` truncate toward zero; `>>` of a negative value is arithmetic;
* pointers are (buffer, element offset, pointee type); multi-dimensional
  arrays are flat; pointer <-> uintptr_t round trips (CONVERT_TO_SHORTPTR /
  CONVERT_TO_BYTEPTR, aom_ports/mem.h:79-80) go through a synthetic address
  map.

Unsupported constructs raise CError at parse or call time (never silently).
"""
import struct as _s
import os
import re

__all__ = ["TU", "CError", "Pointer"]


class CError(Exception):
    pass


# =============================================================================
# types
# =============================================================================
class CType:
    pass


class Void(CType):
    def __repr__(self):
        return "void"


class Int(CType):
    __slots__ = ("bits", "signed", "name", "mask", "half")

    def __init__(self, bits, signed, name):
        self.bits, self.signed, self.name = bits, signed, name
        self.mask = (1 << bits) - 1
        self.half = 1 << (bits - 1)

    def wrap(self, v):
        v &= self.mask
        if self.signed and v >= self.half:
            v -= self.mask + 1
        return v

    def __repr__(self):
        return self.name


class Flt(CType):
    def __init__(self, bits):
        self.bits = bits

    def __repr__(self):
        return "double" if self.bits == 64 else "float"


class Ptr(CType):
    __slots__ = ("to",)

    def __init__(self, to):
        self.to = to

    def __repr__(self):
        return "%r*" % (self.to,)


class Arr(CType):
    __slots__ = ("of", "n")

    def __init__(self, of, n):
        self.of, self.n = of, n

    def __repr__(self):
        return "%r[%s]" % (self.of, self.n)


class Struct(CType):
    def __init__(self, name):
        self.name = name
        self.fields = None  # [(name, type)]
        self.index = {}
        self.is_union = False
        self.packed_unknown = False

    def __repr__(self):
        return "struct %s" % self.name


class Func(CType):
    def __init__(self, ret, params, variadic=False):
        self.ret, self.params, self.variadic = ret, params, variadic

    def __repr__(self):
        return "fn(%s)->%r" % (self.params, self.ret)


VOID = Void()
BOOL = Int(8, False, "_Bool")
CHAR = Int(8, True, "char")
SCHAR = Int(8, True, "signed char")
UCHAR = Int(8, False, "unsigned char")
SHORT = Int(16, True, "short")
USHORT = Int(16, False, "unsigned short")
INT = Int(32, True, "int")
UINT = Int(32, False, "unsigned int")
LONG = Int(64, True, "long")
ULONG = Int(64, False, "unsigned long")
LLONG = Int(64, True, "long long")
ULLONG = Int(64, False, "unsigned long long")
FLOAT = Flt(32)
DOUBLE = Flt(64)

RANK = {8: 1, 16: 2, 32: 3, 64: 4}

BUILTIN_TYPEDEFS = {
    "int8_t": SCHAR, "uint8_t": UCHAR, "int16_t": SHORT, "uint16_t": USHORT,
    "int32_t": INT, "uint32_t": UINT, "int64_t": LONG, "uint64_t": ULONG,
    "intptr_t": LONG, "uintptr_t": ULONG, "size_t": ULONG, "ptrdiff_t": LONG,
    "ssize_t": LONG, "FILE": Struct("FILE"),
    # libc / pthread types the headers mention (system headers are not part of
    # the reference): opaque scalars, never used by the interpreted code paths
    "pthread_mutex_t": LONG, "pthread_cond_t": LONG, "pthread_t": ULONG, "va_list": LONG,
    "jmp_buf": LONG, "pthread_attr_t": LONG, "sem_t": LONG,
    "float_t": FLOAT, "double_t": DOUBLE,  # <math.h> (FLT_EVAL_METHOD 0)
}


def is_int(t):
    return isinstance(t, Int)


def is_arith(t):
    return isinstance(t, (Int, Flt))


def is_ptrlike(t):
    return isinstance(t, (Ptr, Arr))


def decay(t):
    if isinstance(t, Arr):
        return Ptr(t.of)
    if isinstance(t, Func):
        return Ptr(t)
    return t


def promote(t):
    if isinstance(t, Int) and t.bits < 32:
        return INT
    return t


def to_f32(v):
    """Round a Python number to the nearest IEEE single (round-to-nearest-even;
    ints beyond 2^53 rounded directly, not through a double)."""
    if isinstance(v, int) and abs(v) >= (1 << 53):
        import numpy as _np
        return float(_np.float32(_np.int64(v)))  # one correctly rounded cvt
    return _s.unpack("<f", _s.pack("<f", float(v)))[0]


def common_type(a, b):
    # usual arithmetic conversions (C11 6.3.1.8): with a floating operand the
    # result is the wider FLOATING type present; an integer operand converts
    # to it (float + int64 is a float operation)
    if isinstance(a, Flt) or isinstance(b, Flt):
        return DOUBLE if (getattr(a, "bits", 0) == 64 and isinstance(a, Flt)) or \
            (getattr(b, "bits", 0) == 64 and isinstance(b, Flt)) else FLOAT
    a, b = promote(a), promote(b)
    if a.bits == b.bits and a.signed == b.signed:
        return a
    if a.signed == b.signed:
        return a if a.bits > b.bits else b
    u, s = (a, b) if not a.signed else (b, a)
    if u.bits >= s.bits:
        return u
    if s.bits > u.bits:
        return s
    return Int(s.bits, False, "unsigned " + s.name)


def sizeof(t):
    if isinstance(t, Int):
        return t.bits // 8
    if isinstance(t, Flt):
        return t.bits // 8
    if isinstance(t, Ptr):
        return 8
    if isinstance(t, Arr):
        if t.n is None:
            raise CError("sizeof incomplete array")
        return t.n * sizeof(t.of)
    if isinstance(t, Struct):
        if t.packed_unknown:
            raise CError("sizeof a struct with bitfields")
        if t.is_union:
            al = max([alignof(ft) for _, ft in t.fields] or [1])
            sz = max([sizeof(ft) for _, ft in t.fields] or [0])
            return (sz + al - 1) // al * al
        off, al = 0, 1
        for _, ft in t.fields:
            a = alignof(ft)
            off = (off + a - 1) // a * a + sizeof(ft)
            al = max(al, a)
        return (off + al - 1) // al * al
    raise CError("sizeof %r" % (t,))


def alignof(t):
    if isinstance(t, Arr):
        return alignof(t.of)
    if isinstance(t, Struct):
        return max([alignof(ft) for _, ft in t.fields] or [1])
    return sizeof(t)


def slots(t):
    """Flat storage cells an object of type t occupies."""
    if isinstance(t, Arr):
        return (t.n or 0) * slots(t.of)
    return 1


def scalar_of(t):
    while isinstance(t, Arr):
        t = t.of
    return t


# =============================================================================
# runtime values
# =============================================================================
class SObj:
    """A struct object: one cell per field (array fields hold their own flat
    list, struct fields an SObj).  A union keeps one cell per member plus the
    index of the member last accessed; accessing another member first
    re-materialises it from that one's bytes (little-endian layout)."""
    __slots__ = ("st", "vals", "cur")

    def __init__(self, st, vals):
        self.st, self.vals, self.cur = st, vals, 0


def new_storage(t):
    """Flat cells for an object of type t (arrays flattened)."""
    if isinstance(t, Arr):
        inner = scalar_of(t)
        n = slots(t)
        if isinstance(inner, Struct):
            return [new_obj(inner) for _ in range(n)]
        z = 0.0 if isinstance(inner, Flt) else (None if isinstance(inner, Ptr) else 0)
        return [z] * n
    raise CError("new_storage of %r" % (t,))


def new_obj(t):
    """Initial (zero) value of one cell of type t."""
    if isinstance(t, Struct):
        if t.fields is None:
            raise CError("incomplete %r" % (t,))
        return SObj(t, [new_storage(ft) if isinstance(ft, Arr) else new_obj(ft)
                        for _, ft in t.fields])
    if isinstance(t, Flt):
        return 0.0
    if isinstance(t, Ptr):
        return None
    return 0


def copy_obj(v):
    if isinstance(v, SObj):
        o = SObj(v.st, [list(x) if isinstance(x, list) else copy_obj(x) for x in v.vals])
        o.cur = v.cur
        return o
    return v


def to_bytes(v, t):
    """Little-endian object representation (ints, floats, structs, arrays)."""
    import struct as _s
    if isinstance(t, Int):
        return (v & t.mask).to_bytes(t.bits // 8, "little")
    if isinstance(t, Flt):
        return _s.pack("<f" if t.bits == 32 else "<d", v)
    if isinstance(t, Arr):
        es = slots(t.of)
        return b"".join(to_bytes(v[k * es:(k + 1) * es] if isinstance(t.of, Arr) else v[k], t.of)
                        for k in range(t.n))
    if isinstance(t, Struct):
        if t.is_union:
            k = v.cur
            b = to_bytes(v.vals[k], t.fields[k][1])
            return b + bytes(sizeof(t) - len(b))
        out = bytearray()
        for (fn, ft), fv in zip(t.fields, v.vals):
            a = alignof(ft)
            out += bytes((-len(out)) % a)
            out += to_bytes(fv, ft)
        out += bytes((-len(out)) % alignof(t))
        return bytes(out)
    raise CError("object representation of %r" % (t,))


def from_bytes(b, t):
    import struct as _s
    if isinstance(t, Int):
        return t.wrap(int.from_bytes(b[:t.bits // 8], "little"))
    if isinstance(t, Flt):
        return _s.unpack("<f" if t.bits == 32 else "<d", b[:t.bits // 8])[0]
    if isinstance(t, Arr):
        es = sizeof(t.of)
        out = []
        for k in range(t.n):
            x = from_bytes(b[k * es:(k + 1) * es], t.of)
            if isinstance(t.of, Arr):
                out.extend(x)
            else:
                out.append(x)
        return out
    if isinstance(t, Struct):
        o = new_obj(t)
        if t.is_union:
            o.vals[0] = from_bytes(b, t.fields[0][1])
            o.cur = 0
            return o
        off = 0
        for k, (fn, ft) in enumerate(t.fields):
            a = alignof(ft)
            off += (-off) % a
            o.vals[k] = from_bytes(b[off:off + sizeof(ft)], ft)
            off += sizeof(ft)
        return o
    raise CError("object representation of %r" % (t,))


def union_member(obj, idx):
    """Make member idx of a union object current (re-interpreting the bytes
    of the member last accessed)."""
    if obj.cur != idx:
        st = obj.st
        raw = to_bytes(obj.vals[obj.cur], st.fields[obj.cur][1])
        raw = raw + bytes(max(0, sizeof(st.fields[idx][1]) - len(raw)))
        obj.vals[idx] = from_bytes(raw, st.fields[idx][1])
        obj.cur = idx
    return obj


class Pointer:
    __slots__ = ("buf", "off", "ty")

    def __init__(self, buf, off, ty):
        self.buf, self.off, self.ty = buf, off, ty

    def __repr__(self):
        return "<ptr %r +%d>" % (self.ty, self.off)


class FuncRef:
    def __init__(self, name, tu):
        self.name, self.tu = name, tu

    def __call__(self, *args):
        return self.tu.call(self.name, list(args))


# pointer <-> integer: every buffer converted to an integer gets a synthetic
# base address (64-byte aligned, far apart); integers convert back through it
class AddrMap:
    def __init__(self):
        self.base_of = {}
        self.by_base = []
        self.next = 1 << 32

    def to_int(self, p):
        if p is None:
            return 0
        if isinstance(p, FuncRef):
            raise CError("function pointer to integer")
        if p.buf is None:  # already an integer address (e.g. a tagged pointer)
            return p.off
        k = id(p.buf)
        if k not in self.base_of:
            self.base_of[k] = (self.next, p.buf)
            self.by_base.append((self.next, p.buf))
            self.next += 1 << 32
        base = self.base_of[k][0]
        return base + p.off * sizeof(scalar_of(p.ty) if not isinstance(p.ty, Void) else UCHAR)

    def to_ptr(self, v, ty):
        if v == 0:
            return None
        for base, buf in self.by_base:
            if base <= v < base + (1 << 32):
                es = sizeof(scalar_of(ty)) if not isinstance(ty, Void) else 1
                d = v - base
                if d % es:
                    raise CError("misaligned integer->pointer")
                return Pointer(buf, d // es, ty)
        return Pointer(None, v, ty)  # a wild pointer (e.g. a tagged address)


# =============================================================================
# tokenizer + preprocessor
# =============================================================================
TOK_RE = re.compile(r"""
    (?P<ws>[ \t\r\f\v]+) |
    (?P<nl>\n) |
    (?P<num>(0[xX][0-9a-fA-F]+|\d+\.\d*([eE][+-]?\d+)?|\.\d+([eE][+-]?\d+)?|\d+[eE][+-]?\d+|\d+)[uUlLfF]*) |
    (?P<id>[A-Za-z_]\w*) |
    (?P<str>"(\\.|[^"\\])*") |
    (?P<chr>'(\\.|[^'\\])+') |
    (?P<op>\.\.\.|<<=|>>=|->|\+\+|--|<<|>>|<=|>=|==|!=|&&|\|\||\+=|-=|\*=|/=|%=|&=|\^=|\|=|\#\#|[-+*/%<>=!&|^~?:;,.(){}\[\]\#])
""", re.X)


class Tok:
    __slots__ = ("k", "v", "where", "hs")

    def __init__(self, k, v, where=None, hs=frozenset()):
        self.k, self.v, self.where, self.hs = k, v, where, hs

    def __repr__(self):
        return repr(self.v)


def tokenize(text, fname="?", line=1):
    out = []
    pos = 0
    n = len(text)
    while pos < n:
        m = TOK_RE.match(text, pos)
        if not m:
            raise CError("%s:%d: bad character %r" % (fname, line, text[pos]))
        k = m.lastgroup
        if k == "nl":
            line += 1
        elif k != "ws":
            out.append(Tok(k, m.group(k), (fname, line)))
        pos = m.end()
    return out


def strip_comments(src):
    """Comments -> one space (keeping newlines), string literals kept."""
    def rep(m):
        s = m.group(0)
        if s.startswith("//"):
            return " "
        if s.startswith("/*"):
            return " " + "\n" * s.count("\n")
        return s
    return re.sub(r'//[^\n]*|/\*.*?\*/|"(\\.|[^"\\\n])*"|\'(\\.|[^\'\\\n])+\'', rep, src,
                  flags=re.S)


class Macro:
    def __init__(self, name, params, body, variadic=False):
        self.name, self.params, self.body, self.variadic = name, params, body, variadic


class Preprocessor:
    """#define / #undef / #if-family, function-like macros with # and ##,
    hide sets against recursive expansion.  #include is ignored: the TU lists
    its files explicitly, in dependency order."""

    RTCD_DEFS = {"config/aom_dsp_rtcd.h": "aom_dsp/aom_dsp_rtcd_defs.pl",
                 "config/av1_rtcd.h": "av1/common/av1_rtcd_defs.pl",
                 "config/aom_scale_rtcd.h": "aom_scale/aom_scale_rtcd.pl"}

    def __init__(self, defines, root=None):
        self.macros = {}
        self.root = root
        self.done_rtcd = set()
        for k, v in defines.items():
            self.macros[k] = Macro(k, None, tokenize(str(v)))

    def include(self, rest, fname):
        """Tokens of a quoted #include found under the reference root (its
        guards make repeats empty); generated config/* headers and <system>
        headers are skipped (their content is reference_defines / the rtcd
        name fallback)."""
        m = re.match(r'"([^"]+)"', rest)
        if not m or self.root is None:
            return []
        if m.group(1) in self.RTCD_DEFS:
            # a generated rtcd header: its prelude is the `print <<EOF` block
            # of the *_rtcd_defs.pl it is generated from (build/cmake/rtcd.pl
            # copies it verbatim); the prototypes that follow are not needed
            # (calls resolve to the _c functions)
            if m.group(1) in self.done_rtcd:
                return []
            self.done_rtcd.add(m.group(1))
            with open(os.path.join(self.root, self.RTCD_DEFS[m.group(1)])) as fh:
                pl = fh.read()
            pre = re.search(r"print <<EOF\n(.*?)\nEOF", pl, re.S)
            return self.process(pre.group(1), m.group(1), expand=False) if pre else []
        if m.group(1).startswith("config/"):
            return []
        for base in (self.root, os.path.join(self.root, os.path.dirname(fname))):
            path = os.path.join(base, m.group(1))
            if os.path.isfile(path):
                rel = os.path.relpath(path, self.root)
                with open(path) as fh:
                    return self.process(fh.read(), rel, expand=False)
        return []

    def process(self, text, fname, expand=True):
        text = strip_comments(text)
        # join continuation lines, keeping line numbers for the next line
        lines = text.split("\n")
        toks = []
        done = [0]  # toks[:done] are already macro-expanded

        def pending_expand(ts):
            out = ts[:done[0]] + (self.expand(ts[done[0]:]) if expand or True else ts[done[0]:])
            done[0] = len(out)
            return out
        stack = []  # (parent_active, taken)
        active = True
        ln = 0
        while ln < len(lines):
            start = ln + 1
            line = lines[ln]
            while line.endswith("\\") and ln + 1 < len(lines):
                ln += 1
                line = line[:-1] + " " + lines[ln]
            ln += 1
            s = line.strip()
            if s.startswith("#"):
                m = re.match(r"#\s*(\w+)\s*(.*)", s)
                if not m:
                    continue
                kw, rest = m.group(1), m.group(2)
                if kw in ("if", "ifdef", "ifndef"):
                    if not active:
                        stack.append((False, True))
                        continue
                    if kw == "if":
                        c = self.eval_if(rest, fname, start)
                    else:
                        c = (rest.split()[0] in self.macros) == (kw == "ifdef")
                    stack.append((True, c))
                    active = c
                elif kw == "elif":
                    pa, taken = stack[-1]
                    if pa and not taken:
                        c = self.eval_if(rest, fname, start)
                        stack[-1] = (pa, c)
                        active = c
                    else:
                        active = False
                elif kw == "else":
                    pa, taken = stack[-1]
                    active = pa and not taken
                    stack[-1] = (pa, True)
                elif kw == "endif":
                    pa, _ = stack.pop()
                    active = pa
                elif not active:
                    continue
                elif kw == "define":
                    # what precedes is expanded with the macros as they stand
                    # (a function-local #define ... #undef pair, e.g.
                    # UPDATE_SEARCH_STEP in mcomp.c, must apply in between)
                    toks = pending_expand(toks)
                    self.define(rest, fname, start)
                elif kw == "undef":
                    toks = pending_expand(toks)
                    self.macros.pop(rest.split()[0], None)
                elif kw == "error":
                    raise CError("%s:%d: #error %s" % (fname, start, rest))
                elif kw == "include":
                    # expand what precedes with the macros defined so far
                    toks = pending_expand(toks) + self.include(rest, fname)
                    done[0] = len(toks)
                continue
            if active and s:
                toks.extend(tokenize(line, fname, start))
        toks = pending_expand(toks)
        return toks

    def define(self, rest, fname, ln):
        m = re.match(r"(\w+)", rest)
        name = m.group(1)
        after = rest[len(name):]
        if after.startswith("("):
            close = after.index(")")
            ps = [p.strip() for p in after[1:close].split(",") if p.strip()]
            variadic = bool(ps) and ps[-1] == "..."
            if variadic:
                ps[-1] = "__VA_ARGS__"
            self.macros[name] = Macro(name, ps, tokenize(after[close + 1:], fname, ln), variadic)
        else:
            self.macros[name] = Macro(name, None, tokenize(after, fname, ln))

    def eval_if(self, expr, fname, ln):
        expr = re.sub(r"defined\s*\(\s*(\w+)\s*\)|defined\s+(\w+)",
                      lambda m: "1" if (m.group(1) or m.group(2)) in self.macros else "0", expr)
        py = []
        for t in self.expand(tokenize(expr, fname, ln)):
            if t.k == "id":
                py.append(" 0 ")
            elif t.k == "num":
                py.append(" %d " % int(t.v.rstrip("uUlL"), 0))
            elif t.v == "&&":
                py.append(" and ")
            elif t.v == "||":
                py.append(" or ")
            elif t.v == "!":
                py.append(" not ")
            elif t.v == "/":
                py.append("//")
            else:
                py.append(t.v)
        try:
            return bool(eval("".join(py), {}, {}))
        except Exception as e:
            raise CError("%s:%d: cannot evaluate #if %s (%s)" % (fname, ln, expr, e))

    def expand(self, toks):
        work = list(reversed(toks))
        out = []
        while work:
            t = work.pop()
            if t.k == "id" and t.v in self.macros and t.v not in t.hs:
                m = self.macros[t.v]
                hs = t.hs | {t.v}
                if m.params is None:
                    work.extend(reversed([Tok(x.k, x.v, t.where, x.hs | hs) for x in m.body]))
                    continue
                if work and work[-1].v == "(":
                    args = self.collect_args(work)
                    body = self.substitute(m, args)
                    work.extend(reversed([Tok(x.k, x.v, t.where, x.hs | hs) for x in body]))
                    continue
            out.append(t)
        return out

    @staticmethod
    def collect_args(work):
        work.pop()  # '('
        depth = 1
        args, cur = [], []
        while True:
            t = work.pop()
            if t.v == "(":
                depth += 1
            elif t.v == ")":
                depth -= 1
                if depth == 0:
                    args.append(cur)
                    return args
            elif t.v == "," and depth == 1:
                args.append(cur)
                cur = []
                continue
            cur.append(t)

    def substitute(self, m, args):
        params = m.params
        if m.variadic:
            nfix = len(params) - 1
            va = []
            for k, a in enumerate(args[nfix:]):
                if k:
                    va.append(Tok("op", ","))
                va.extend(a)
            args = args[:nfix] + [va]
        if not params and args == [[]]:
            args = []
        if len(args) != len(params):
            raise CError("macro %s: %d args for %d params" % (m.name, len(args), len(params)))
        amap = dict(zip(params, args))
        body = m.body
        out = []
        k = 0
        while k < len(body):
            t = body[k]
            if t.v == "#" and k + 1 < len(body) and body[k + 1].v in amap:
                out.append(Tok("str", '"%s"' % " ".join(x.v for x in amap[body[k + 1].v])))
                k += 2
                continue
            if t.v == "##" and k + 1 < len(body):
                nt = body[k + 1]
                rep = list(amap[nt.v]) if (nt.k == "id" and nt.v in amap) else [nt]
                if rep:
                    left = out.pop() if out else None
                    merged = tokenize((left.v if left else "") + rep[0].v)
                    out.extend(merged)
                    out.extend(rep[1:])
                k += 2
                continue
            if t.k == "id" and t.v in amap:
                raw = k + 1 < len(body) and body[k + 1].v == "##"
                out.extend(amap[t.v] if raw else self.expand(amap[t.v]))
            else:
                out.append(Tok(t.k, t.v, t.where))
            k += 1
        return out


# =============================================================================
# parser (C subset) -> AST tuples
# =============================================================================
TYPE_KW = {"void", "char", "short", "int", "long", "signed", "unsigned", "float", "double",
           "_Bool", "struct", "union", "enum"}
QUAL_KW = {"const", "volatile", "restrict", "__restrict", "__restrict__", "static", "extern",
           "inline", "__inline", "__inline__", "register", "typedef", "auto", "_Noreturn",
           "__extension__"}


class Parser:
    _anon = 0

    def __init__(self, toks, scope):
        self.t = toks
        self.i = 0
        self.sc = scope  # TU: typedefs, structs, enums

    # ---- token helpers ----
    def peek(self, k=0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else Tok("eof", "<eof>")

    def next(self):
        t = self.peek()
        self.i += 1
        return t

    def accept(self, v):
        if self.peek().v == v and self.peek().k != "str":
            self.i += 1
            return True
        return False

    def expect(self, v):
        t = self.next()
        if t.v != v:
            raise CError("expected %r, got %r at %s" % (v, t.v, t.where))
        return t

    def skip_attr(self):
        while self.peek().v in ("__attribute__", "__declspec", "__asm__", "asm"):
            self.next()
            self.expect("(")
            d = 1
            while d:
                t = self.next()
                if t.v == "(":
                    d += 1
                elif t.v == ")":
                    d -= 1

    def is_type_start(self, k=0):
        t = self.peek(k)
        if t.k != "id":
            return False
        return (t.v in TYPE_KW or t.v in QUAL_KW or t.v in self.sc.typedefs
                or t.v in ("__attribute__",))

    # ---- declarations ----
    def decl_specs(self):
        """-> (base type, storage dict)"""
        st = {"typedef": False, "static": False, "extern": False}
        words = []
        base = None
        while True:
            self.skip_attr()
            t = self.peek()
            if t.k != "id":
                break
            if t.v in QUAL_KW:
                self.next()
                if t.v in st:
                    st[t.v] = True
                continue
            if t.v in ("struct", "union"):
                self.next()
                base = self.struct_spec(t.v)
                continue
            if t.v == "enum":
                self.next()
                base = self.enum_spec()
                continue
            if t.v in TYPE_KW:
                words.append(self.next().v)
                continue
            if t.v in self.sc.typedefs and base is None and not words:
                self.next()
                base = self.sc.typedefs[t.v]
                continue
            break
        if base is None:
            if not words:
                raise CError("expected a type at %s (%r)" % (self.peek().where, self.peek().v))
            base = self.int_type(words)
        return base, st

    def int_type(self, words):
        w = sorted(words)
        if "void" in w:
            return VOID
        if "float" in w:
            return FLOAT
        if "double" in w:
            return DOUBLE
        if "_Bool" in w:
            return BOOL
        uns = "unsigned" in w
        if "char" in w:
            return UCHAR if uns else (SCHAR if "signed" in w else CHAR)
        if "short" in w:
            return USHORT if uns else SHORT
        nl = w.count("long")
        if nl >= 1:
            return (ULLONG if uns else LLONG) if nl == 2 else (ULONG if uns else LONG)
        return UINT if uns else INT

    def struct_spec(self, kind):
        self.skip_attr()
        name = None
        if self.peek().k == "id":
            name = self.next().v
        Parser._anon += 1
        key = (kind + " " + name) if name else ("<anon%d>" % Parser._anon)
        st = self.sc.structs.get(key)
        if st is None:
            st = Struct(key)
            st.is_union = kind == "union"
            if name:
                self.sc.structs[key] = st
        if self.accept("{"):
            fields = []
            while not self.accept("}"):
                base, _ = self.decl_specs()
                while True:
                    if self.peek().v == ":":  # unnamed bitfield (padding)
                        self.next()
                        self.sc.const_eval(self.cond_expr())
                        if not self.accept(","):
                            break
                        continue
                    fname, ftype = self.declarator(base)
                    if self.accept(":"):
                        # a bitfield: an integer of that width (stores wrap
                        # to it); layout is not modelled (no sizeof use)
                        width = self.sc.const_eval(self.cond_expr())
                        ftype = Int(width, ftype.signed, "%s:%d" % (ftype.name, width))
                        st.packed_unknown = True
                    fields.append((fname, ftype))
                    if not self.accept(","):
                        break
                self.expect(";")
            st.fields = fields
            st.index = {f: k for k, (f, _) in enumerate(fields)}
        return st

    def enum_spec(self):
        self.skip_attr()
        if self.peek().k == "id":
            self.next()
        if self.accept("{"):
            val = 0
            while not self.accept("}"):
                nm = self.next().v
                if self.accept("="):
                    e = self.assign_expr(no_comma=True)
                    val = self.sc.const_eval(e)
                self.sc.enums[nm] = val
                val += 1
                if not self.accept(","):
                    self.expect("}")
                    break
        return INT

    def declarator(self, base, abstract=False):
        """-> (name, type).  Handles pointers, arrays, function params and
        parenthesised declarators."""
        ptrs = 0
        while True:
            self.skip_attr()
            if self.accept("*"):
                ptrs += 1
                while self.peek().v in ("const", "volatile", "restrict", "__restrict",
                                        "__restrict__"):
                    self.next()
                continue
            break
        name = None
        inner = None
        if self.peek().v == "(" and (self.peek(1).v == "*" or (self.peek(1).k == "id" and not
                                                               self.is_type_start(1)
                                                               and self.peek(2).v == ")")):
            self.next()
            inner = self.i
            # skip the inner declarator for now; parse suffixes first
            d = 1
            while d:
                t = self.next()
                if t.v == "(":
                    d += 1
                elif t.v == ")":
                    d -= 1
            inner_end = self.i
        elif self.peek().k == "id" and not self.is_type_start():
            name = self.next().v
        self.skip_attr()
        t = base
        for _ in range(ptrs):
            t = Ptr(t)
        suffixes = []
        while True:
            if self.accept("["):
                if self.accept("]"):
                    suffixes.append(("arr", None))
                else:
                    while self.peek().v in ("const", "static", "restrict"):
                        self.next()
                    e = self.assign_expr()
                    self.expect("]")
                    suffixes.append(("arr", self.sc.const_eval(e)))
                continue
            if self.peek().v == "(":
                self.next()
                params, variadic = self.param_list()
                suffixes.append(("fn", params, variadic))
                continue
            break
        for s in reversed(suffixes):
            if s[0] == "arr":
                t = Arr(t, s[1])
            else:
                t = Func(t, s[1], s[2])
        self.skip_attr()
        if inner is not None:
            save = self.i
            self.i = inner
            name, t = self.declarator(t, abstract)
            self.expect(")")
            self.i = save
        if isinstance(t, Func) and not hasattr(t, "names"):
            t.names = getattr(self, "_last_param_names", None)
        return name, t

    def param_list(self):
        params, names = [], []
        variadic = False
        if self.accept(")"):
            self._last_param_names = names
            return params, variadic
        if self.peek().v == "void" and self.peek(1).v == ")":
            self.next()
            self.next()
            self._last_param_names = names
            return params, variadic
        while True:
            if self.accept("..."):
                variadic = True
                break
            base, _ = self.decl_specs()
            nm, t = self.declarator(base, abstract=True)
            if isinstance(t, Arr):
                t = Ptr(t.of)
            elif isinstance(t, Func):
                t = Ptr(t)
            params.append(t)
            names.append(nm)
            if not self.accept(","):
                break
        self.expect(")")
        self._last_param_names = names
        return params, variadic

    def type_name(self):
        base, _ = self.decl_specs()
        _, t = self.declarator(base, abstract=True)
        return t

    # ---- initialisers ----
    def initializer(self):
        if self.accept("{"):
            items = []
            while not self.accept("}"):
                desig = None
                if self.peek().v == "." and self.peek(1).k == "id":
                    self.next()
                    desig = ("field", self.next().v)
                    self.expect("=")
                elif self.peek().v == "[":
                    self.next()
                    desig = ("index", self.sc.const_eval(self.assign_expr()))
                    self.expect("]")
                    self.expect("=")
                items.append((desig, self.initializer()))
                if not self.accept(","):
                    self.expect("}")
                    break
            return ("init_list", items)
        return self.assign_expr()

    # ---- statements ----
    def compound(self):
        self.expect("{")
        items = []
        while not self.accept("}"):
            items.append(self.block_item())
        return ("block", items)

    def block_item(self):
        if self.is_decl_start():
            return self.declaration(local=True)
        return self.statement()

    def is_decl_start(self):
        t = self.peek()
        if t.k != "id":
            return False
        if t.v in TYPE_KW or t.v in QUAL_KW:
            return True
        if t.v in self.sc.typedefs:
            # "T x" / "T *x" (not an expression "T * x" -- typedef names are
            # never variables in this code)
            return self.peek(1).v != "=" and self.peek(1).v != "(" or self.peek(1).v == "("
        return False

    def declaration(self, local):
        base, st = self.decl_specs()
        decls = []
        if self.accept(";"):
            return ("decl", decls, st)
        while True:
            name, t = self.declarator(base)
            init = None
            if self.accept("="):
                init = self.initializer()
            if st["typedef"]:
                self.sc.typedefs[name] = t
            else:
                decls.append((name, t, init))
            if not self.accept(","):
                break
        self.expect(";")
        return ("decl", decls, st)

    def statement(self):
        t = self.peek()
        v = t.v
        if v == "{":
            return self.compound()
        if t.k == "id":
            if v == "if":
                self.next()
                self.expect("(")
                c = self.expr()
                self.expect(")")
                a = self.statement()
                b = self.statement() if self.accept("else") else None
                return ("if", c, a, b)
            if v == "for":
                self.next()
                self.expect("(")
                init = None
                if not self.accept(";"):
                    if self.is_decl_start():
                        init = self.declaration(local=True)
                    else:
                        init = ("expr", self.expr())
                        self.expect(";")
                cond = None if self.peek().v == ";" else self.expr()
                self.expect(";")
                step = None if self.peek().v == ")" else self.expr()
                self.expect(")")
                body = self.statement()
                return ("for", init, cond, step, body)
            if v == "while":
                self.next()
                self.expect("(")
                c = self.expr()
                self.expect(")")
                return ("while", c, self.statement())
            if v == "do":
                self.next()
                body = self.statement()
                self.expect("while")
                self.expect("(")
                c = self.expr()
                self.expect(")")
                self.expect(";")
                return ("do", body, c)
            if v == "return":
                self.next()
                e = None if self.peek().v == ";" else self.expr()
                self.expect(";")
                return ("return", e)
            if v == "break":
                self.next()
                self.expect(";")
                return ("break",)
            if v == "continue":
                self.next()
                self.expect(";")
                return ("continue",)
            if v == "switch":
                self.next()
                self.expect("(")
                c = self.expr()
                self.expect(")")
                return ("switch", c, self.statement())
            if v == "case":
                self.next()
                e = self.cond_expr()
                self.expect(":")
                return ("case", self.sc.const_eval(e))
            if v == "default" and self.peek(1).v == ":":
                self.next()
                self.next()
                return ("default",)
            if v == "goto":
                raise CError("goto unsupported")
        if self.accept(";"):
            return ("nop",)
        e = self.expr()
        self.expect(";")
        return ("expr", e)

    # ---- expressions ----
    def expr(self):
        e = self.assign_expr()
        while self.accept(","):
            e = ("comma", e, self.assign_expr())
        return e

    ASSIGN_OPS = {"=", "+=", "-=", "*=", "/=", "%=", "<<=", ">>=", "&=", "^=", "|="}

    def assign_expr(self, no_comma=True):
        lhs = self.cond_expr()
        t = self.peek()
        if t.k == "op" and t.v in self.ASSIGN_OPS:
            self.next()
            rhs = self.assign_expr()
            return ("assign", t.v, lhs, rhs)
        return lhs

    def cond_expr(self):
        c = self.binary(0)
        if self.accept("?"):
            a = self.expr()
            self.expect(":")
            b = self.cond_expr()
            return ("cond", c, a, b)
        return c

    BINOPS = [["||"], ["&&"], ["|"], ["^"], ["&"], ["==", "!="], ["<", ">", "<=", ">="],
              ["<<", ">>"], ["+", "-"], ["*", "/", "%"]]

    def binary(self, lvl):
        if lvl == len(self.BINOPS):
            return self.cast_expr()
        e = self.binary(lvl + 1)
        while True:
            t = self.peek()
            if t.k == "op" and t.v in self.BINOPS[lvl]:
                self.next()
                e = ("bin", t.v, e, self.binary(lvl + 1))
            else:
                return e

    def cast_expr(self):
        if self.peek().v == "(" and self.is_type_start(1):
            save = self.i
            self.next()
            t = self.type_name()
            self.expect(")")
            if self.peek().v == "{":
                raise CError("compound literals unsupported")
            return ("cast", t, self.cast_expr())
        return self.unary()

    def unary(self):
        t = self.peek()
        if t.k == "op":
            if t.v in ("++", "--"):
                self.next()
                return ("preinc", t.v, self.unary())
            if t.v in ("-", "+", "!", "~", "*", "&"):
                self.next()
                return ("un", t.v, self.cast_expr())
        if t.v == "sizeof" and t.k == "id":
            self.next()
            if self.peek().v == "(" and self.is_type_start(1):
                self.next()
                ty = self.type_name()
                self.expect(")")
                return ("sizeof_t", ty)
            return ("sizeof_e", self.unary())
        return self.postfix()

    def postfix(self):
        e = self.primary()
        while True:
            t = self.peek()
            if t.v == "[":
                self.next()
                i = self.expr()
                self.expect("]")
                e = ("index", e, i)
            elif t.v == "(":
                self.next()
                args = []
                if not self.accept(")"):
                    while True:
                        args.append(self.assign_expr())
                        if not self.accept(","):
                            break
                    self.expect(")")
                e = ("call", e, args)
            elif t.v == ".":
                self.next()
                e = ("member", e, self.next().v)
            elif t.v == "->":
                self.next()
                e = ("arrow", e, self.next().v)
            elif t.v in ("++", "--") and t.k == "op":
                self.next()
                e = ("postinc", t.v, e)
            else:
                return e

    def primary(self):
        t = self.next()
        if t.k == "num":
            return ("num", t.v)
        if t.k == "chr":
            s = t.v[1:-1]
            if s.startswith("\\"):
                s = bytes(s, "ascii").decode("unicode_escape")
            return ("numv", ord(s), INT)
        if t.k == "str":
            s = t.v
            while self.peek().k == "str":
                s = s[:-1] + self.next().v[1:]
            return ("str", s)
        if t.k == "id":
            return ("id", t.v)
        if t.v == "(":
            e = self.expr()
            self.expect(")")
            return e
        raise CError("unexpected %r at %s" % (t.v, t.where))


def num_const(text):
    s = text
    low = s.lower()
    if ("." in s or ("e" in low and not low.startswith("0x"))) or (low.endswith("f") and not low.startswith("0x")):
        v = float(s.rstrip("fFlL"))
        if low.endswith("f"):
            return to_f32(v), FLOAT
        return v, DOUBLE
    suf = ""
    while s and s[-1] in "uUlL":
        suf = s[-1].lower() + suf
        s = s[:-1]
    v = int(s, 0)
    uns = "u" in suf
    lng = "l" in suf
    hexoct = s.startswith("0") and len(s) > 1
    cands = []
    if not lng:
        cands += [INT] if not uns else [UINT]
        if hexoct and not uns:
            cands += [UINT]
    cands += [LONG] if not uns else [ULONG]
    if hexoct or uns:
        cands += [ULONG]
    for c in cands:
        lo = -(1 << (c.bits - 1)) if c.signed else 0
        hi = (1 << (c.bits - 1)) - 1 if c.signed else (1 << c.bits) - 1
        if lo <= v <= hi:
            return v, c
    return v, ULONG


# =============================================================================
# compiler: AST -> Python closures over a per-call frame list
# =============================================================================
BRK, CONT, RET = 1, 2, 3


class FuncScope:
    def __init__(self):
        self.nslots = 1  # slot 0: return value
        self.scopes = [{}]

    def lookup(self, name):
        for s in reversed(self.scopes):
            if name in s:
                return s[name]
        return None

    def add(self, name, t):
        k = self.nslots
        self.nslots += 1
        self.scopes[-1][name] = (k, t)
        return k


class TU:
    """A set of reference source files, preprocessed and parsed together."""

    def __init__(self, root, files, defines):
        self.root = root
        self.typedefs = dict(BUILTIN_TYPEDEFS)
        self.structs = {}
        self.enums = {}
        self.func_defs = {}    # name -> (Func type, param names, body)
        self.func_decls = {}   # name -> Func type
        self.global_defs = {}  # name -> (type, init)
        self.globals = {}      # name -> (cell list, index, type) once initialised
        self.compiled = {}
        self.addr = AddrMap()
        self.errors = []
        self.pp = Preprocessor(defines, root)
        for f in files:
            with open(os.path.join(root, f)) as fh:
                toks = self.pp.process(fh.read(), f)
            self.parse_top(toks, f)

    def add_source(self, text, fname):
        """Parse extra C text in this TU (e.g. a wrapper around a fragment of a
        reference function body, read from the reference at run time)."""
        self.parse_top(self.pp.process(text, fname), fname)

    # ---- top level ----
    def parse_top(self, toks, fname):
        i = 0
        n = len(toks)
        while i < n:
            # one external declaration: up to ';' at depth 0 or a function body
            j = i
            depth = 0
            end = None
            while j < n:
                v = toks[j].v
                if v in ("(", "["):
                    depth += 1
                elif v in (")", "]"):
                    depth -= 1
                elif v == "{":
                    if depth == 0 and toks[j - 1].v == ")" and "=" not in [t.v for t in toks[i:j]] \
                            and not self._attr_paren(toks, j - 1):
                        # function body: match braces
                        d = 0
                        k = j
                        while True:
                            if toks[k].v == "{":
                                d += 1
                            elif toks[k].v == "}":
                                d -= 1
                                if d == 0:
                                    break
                            k += 1
                        end = k + 1
                        break
                    depth += 1
                elif v == "}":
                    depth -= 1
                elif v == ";" and depth == 0:
                    end = j + 1
                    break
                j += 1
            if end is None:
                end = n
            chunk = toks[i:end]
            i = end
            if not chunk or (len(chunk) == 1 and chunk[0].v == ";"):
                continue
            if chunk[0].v == "extern" and len(chunk) > 1 and chunk[1].k == "str":
                # extern "C" { ... }: not in C sources
                continue
            try:
                self.parse_external(chunk)
            except CError as e:
                self.errors.append((fname, chunk[0].where, str(e)))
            except (IndexError, KeyError, AttributeError, TypeError, ValueError) as e:
                self.errors.append((fname, chunk[0].where, repr(e)))

    @staticmethod
    def _attr_paren(toks, close):
        """True when the ')' at toks[close] ends an __attribute__((...))."""
        d = 0
        k = close
        while k >= 0:
            if toks[k].v == ")":
                d += 1
            elif toks[k].v == "(":
                d -= 1
                if d == 0:
                    break
            k -= 1
        while k > 0 and toks[k - 1].v == "(":
            k -= 1
        return k > 0 and toks[k - 1].v in ("__attribute__", "__declspec")

    def parse_external(self, chunk):
        p = Parser(chunk + [Tok("eof", "<eof>")], self)
        base, st = p.decl_specs()
        if p.accept(";"):
            return
        while True:
            name, t = p.declarator(base)
            if isinstance(t, Func) and p.peek().v == "{":
                body = p.compound()
                self.func_defs[name] = (t, t.names, body)
                return
            init = None
            if p.accept("="):
                init = p.initializer()
            if st["typedef"]:
                self.typedefs[name] = t
            elif isinstance(t, Func):
                self.func_decls[name] = t
            elif not (st["extern"] and init is None):
                self.global_defs[name] = (t, init)
            elif name not in self.global_defs:
                self.global_defs.setdefault("__extern__" + name, (t, None))
            if not p.accept(","):
                break
        p.expect(";")

    # ---- constants ----
    def const_eval(self, e):
        k = e[0]
        if k == "num":
            return num_const(e[1])[0]
        if k == "numv":
            return e[1]
        if k == "id":
            if e[1] in self.enums:
                return self.enums[e[1]]
            raise CError("not a constant: %s" % e[1])
        if k == "un":
            v = self.const_eval(e[2])
            return {"-": -v, "+": v, "~": ~v, "!": int(not v)}[e[1]]
        if k == "bin":
            a, b = self.const_eval(e[2]), self.const_eval(e[3])
            op = e[1]
            if op == "/":
                return int(a / b) if b else 0
            if op == "%":
                return a - int(a / b) * b
            return int(eval("a %s b" % {"&&": "and", "||": "or"}.get(op, op)))
        if k == "cond":
            return self.const_eval(e[2]) if self.const_eval(e[1]) else self.const_eval(e[3])
        if k == "cast":
            v = self.const_eval(e[2])
            return e[1].wrap(v) if isinstance(e[1], Int) else v
        if k == "sizeof_t":
            return sizeof(e[1])
        if k == "sizeof_e":
            return sizeof(self.static_type(e[1]))
        raise CError("not a constant expression: %r" % (e,))

    def static_type(self, e):
        if e[0] == "id":
            g = self.global_type(e[1])
            if g is not None:
                return g
        if e[0] == "index":
            t = self.static_type(e[1])
            return t.of if isinstance(t, Arr) else t.to
        raise CError("sizeof expression unsupported: %r" % (e,))

    # ---- globals ----
    def global_type(self, name):
        if name in self.global_defs:
            return self.global_defs[name][0]
        return None

    def global_cell(self, name):
        g = self.globals.get(name)
        if g is not None:
            return g
        if name not in self.global_defs:
            return None
        t, init = self.global_defs[name]
        if isinstance(t, Arr) and t.n is None:
            if init is None or init[0] != "init_list":
                raise CError("incomplete array %s" % name)
            t = Arr(t.of, self.init_count(t, init))
            self.global_defs[name] = (t, init)
        if isinstance(t, Arr):
            cell = new_storage(t)
            g = (cell, 0, t)
        else:
            cell = [new_obj(t)]
            g = (cell, 0, t)
        self.globals[name] = g
        if init is not None:
            fs = FuncScope()
            self.store_init(fs, t, init)(cell, 0, [None])
        return g

    def init_count(self, t, init):
        items = init[1]
        if isinstance(t.of, Arr) or isinstance(t.of, Struct):
            if all(isinstance(x[1], tuple) and x[1][0] == "init_list" for x in items):
                return len(items)
            return -(-len(items) // slots(t.of))
        return len(items)

    # ---- initialiser compilation ----
    def store_init(self, fs, t, init):
        """-> fn(buf, off, frame) storing the initialiser into an object of
        type t at buf[off] (flat)."""
        if init[0] != "init_list":
            if isinstance(t, Arr) and init[0] == "str":
                raise CError("string initialisers unsupported")
            f, et = self.rvalue(fs, init)
            conv = self.converter(et, t)

            def st(buf, off, fr):
                buf[off] = conv(f(fr))
            return st
        items = init[1]
        if isinstance(t, Struct):
            ops = []
            fi = 0
            for desig, it in items:
                if desig and desig[0] == "field":
                    fi = t.index[desig[1]]
                fname, ft = t.fields[fi]
                ops.append((fi, ft, self.store_init(fs, ft, it)))
                fi += 1

            def st(buf, off, fr):
                obj = buf[off]
                for k, ft, s in ops:
                    if isinstance(ft, Arr):
                        s(obj.vals[k], 0, fr)
                    else:
                        s(obj.vals, k, fr)
            return st
        if isinstance(t, Arr):
            el = t.of
            es = slots(el)
            ops = []
            idx = 0
            k = 0
            # brace elision: scalars filling sub-aggregates in order
            flat_mode = isinstance(el, (Arr, Struct)) and not all(
                isinstance(x[1], tuple) and x[1][0] == "init_list" for x in items)
            if flat_mode:
                inner = scalar_of(t)
                for n_, (desig, it) in enumerate(items):
                    ops.append((n_, self.store_init(fs, inner, it)))

                def st(buf, off, fr):
                    for pos, s in ops:
                        s(buf, off + pos, fr)
                return st
            for desig, it in items:
                if desig and desig[0] == "index":
                    idx = desig[1]
                ops.append((idx * es, self.store_init(fs, el, it)))
                idx += 1

            def st(buf, off, fr):
                for pos, s in ops:
                    s(buf, off + pos, fr)
            return st
        # scalar in braces
        if len(items) != 1:
            raise CError("scalar initialiser list")
        return self.store_init(fs, t, items[0][1])

    # ---- functions ----
    def has_func(self, name):
        return name in self.func_defs or (name + "_c") in self.func_defs

    def resolve_name(self, name):
        if name in self.func_defs:
            return name
        if name + "_c" in self.func_defs:  # rtcd.pl single-impl: #define f f_c
            return name + "_c"
        return None

    def func(self, name):
        rn = self.resolve_name(name)
        if rn is None:
            raise CError("no definition of %s" % name)
        return FuncRef(rn, self)

    def call(self, name, args):
        fn = self.compiled.get(name)
        if fn is None:
            fn = self.compile_func(name)
        return fn(args)

    def compile_func(self, name):
        ft, names, body = self.func_defs[name]
        fs = FuncScope()
        fs.ret = ft.ret
        pslots = []
        for pn, pt in zip(names, ft.params):
            pslots.append((fs.add(pn, pt), pt))
        holder = {}

        def call(args, _holder=holder):
            return _holder["f"](args)
        self.compiled[name] = call  # recursion
        bodyf = self.stmt(fs, body)
        nslots = [0]
        convs = [(k, self.converter(None, pt)) for k, pt in pslots]
        ret_void = isinstance(ft.ret, Void)

        def run(args):
            fr = [None] * nslots[0]
            if len(args) != len(convs):
                raise CError("%s: %d args for %d params" % (name, len(args), len(convs)))
            for (k, cv), a in zip(convs, args):
                fr[k] = cv(a)
            bodyf(fr)
            return None if ret_void else fr[0]
        nslots[0] = fs.nslots
        holder["f"] = run
        self.compiled[name] = run
        return run

    # ---- conversions ----
    def converter(self, src, dst):
        """value of type src -> value of type dst (assignment / cast)."""
        if isinstance(dst, Int):
            if isinstance(src, Flt):
                return lambda v: dst.wrap(int(v))
            if isinstance(src, (Ptr, Arr)):
                return lambda v: dst.wrap(self.addr.to_int(v))
            if dst is BOOL or dst.name == "_Bool":
                return lambda v: 1 if v else 0
            return dst.wrap
        if isinstance(dst, Flt):
            if dst.bits == 32:
                return to_f32
            return float
        if isinstance(dst, Ptr):
            if isinstance(src, Int):
                def cv(v):
                    if v is None or isinstance(v, Pointer):
                        return v
                    return self.addr.to_ptr(v, dst.to)
                return cv

            def cvp(v):
                if isinstance(v, Pointer) and v.ty is not dst.to and not isinstance(dst.to, Void):
                    if v.buf is None:
                        return self.addr.to_ptr(v.off, dst.to) if False else Pointer(None, v.off, dst.to)
                    return Pointer(v.buf, v.off, dst.to)
                return v
            return cvp
        if isinstance(dst, Struct):
            return copy_obj
        return lambda v: v

    # ---- lvalues: fn(frame) -> (buf, off); arrays: flat storage start ----
    def lvalue(self, fs, e):
        k = e[0]
        if k == "id":
            name = e[1]
            loc = fs.lookup(name)
            if loc is not None:
                slot, t = loc
                if isinstance(t, Arr):
                    return (lambda fr: (fr[slot], 0)), t
                return (lambda fr: (fr, slot)), t
            g = self.global_cell(name)
            if g is not None:
                cell, off, t = g
                if isinstance(t, Arr):
                    return (lambda fr: (cell, 0)), t
                return (lambda fr: (cell, 0)), t
            raise CError("unknown identifier %s" % name)
        if k == "index":
            bf, bt = self.rvalue(fs, e[1])
            xf, xt = self.rvalue(fs, e[2])
            if is_int(bt) and isinstance(xt, Ptr):
                bf, bt, xf, xt = xf, xt, bf, bt
            if not isinstance(bt, Ptr):
                raise CError("subscript of %r" % (bt,))
            el = bt.to
            es = slots(el)
            def loc(fr):
                p = bf(fr)
                o = p.off + xf(fr) * es
                if o < 0 or p.buf is None:
                    raise CError("out-of-bounds / wild access at offset %d" % o)
                return p.buf, o
            return loc, el
        if k == "un" and e[1] == "*":
            pf, pt = self.rvalue(fs, e[2])
            if not isinstance(pt, Ptr):
                raise CError("deref of %r" % (pt,))

            def loc(fr):
                p = pf(fr)
                if p.buf is None:
                    p = self.addr.to_ptr(p.off, p.ty)
                    if p.buf is None:
                        raise CError("dereference of a wild pointer")
                if p.off < 0:
                    raise CError("out-of-bounds access at offset %d" % p.off)
                return p.buf, p.off
            return loc, pt.to
        if k in ("member", "arrow"):
            if k == "member":
                sf, stt = self.lvalue(fs, e[1])
                getobj = lambda fr: (lambda b: b[0][b[1]])(sf(fr))
            else:
                pf, pt = self.rvalue(fs, e[1])
                stt = pt.to
                getobj = lambda fr: (lambda p: p.buf[p.off])(pf(fr))
            if not isinstance(stt, Struct) or stt.fields is None:
                raise CError("member of %r" % (stt,))
            idx = stt.index[e[2]]
            ft = stt.fields[idx][1]
            if stt.is_union:
                if isinstance(ft, Arr):
                    return (lambda fr: (union_member(getobj(fr), idx).vals[idx], 0)), ft
                return (lambda fr: (union_member(getobj(fr), idx).vals, idx)), ft
            if isinstance(ft, Arr):
                return (lambda fr: (getobj(fr).vals[idx], 0)), ft
            return (lambda fr: (getobj(fr).vals, idx)), ft
        raise CError("not an lvalue: %r" % (k,))

    # ---- rvalues: fn(frame) -> value, type ----
    def rvalue(self, fs, e):
        f, t = self._rvalue(fs, e)
        return f, t

    def _rvalue(self, fs, e):
        k = e[0]
        if k == "num":
            v, t = num_const(e[1])
            return (lambda fr: v), t
        if k == "numv":
            v = e[1]
            return (lambda fr: v), e[2]
        if k == "str":
            s = e[1]
            return (lambda fr: s), Ptr(CHAR)
        if k == "id":
            name = e[1]
            if fs.lookup(name) is None:
                if name in self.enums:
                    v = self.enums[name]
                    return (lambda fr: v), INT
                if self.global_type(name) is None:
                    rn = self.resolve_name(name)
                    if rn is not None:
                        ref = FuncRef(rn, self)
                        return (lambda fr: ref), Ptr(self.func_defs[rn][0])
                    if name == "NULL":
                        return (lambda fr: None), Ptr(VOID)
                    raise CError("unknown identifier %s" % name)
            return self.load(fs, e)
        if k in ("index", "member", "arrow") or (k == "un" and e[1] == "*"):
            return self.load(fs, e)
        if k == "un":
            return self.unop(fs, e)
        if k == "bin":
            return self.binop(fs, e)
        if k == "assign":
            return self.assign(fs, e)
        if k in ("preinc", "postinc"):
            return self.incdec(fs, e)
        if k == "cast":
            f, st = self.rvalue(fs, e[2])
            if isinstance(e[1], Void):
                return (lambda fr: (f(fr), None)[1]), VOID
            cv = self.converter(st, e[1])
            return (lambda fr: cv(f(fr))), e[1]
        if k == "cond":
            cf, ct = self.rvalue(fs, e[1])
            af, at = self.rvalue(fs, e[2])
            bf, bt = self.rvalue(fs, e[3])
            if is_arith(at) and is_arith(bt):
                rt = common_type(at, bt)
                ca, cb = self.converter(at, rt), self.converter(bt, rt)
                return (lambda fr: ca(af(fr)) if cf(fr) else cb(bf(fr))), rt
            rt = at if isinstance(at, Ptr) else bt
            return (lambda fr: af(fr) if cf(fr) else bf(fr)), rt
        if k == "comma":
            af, _ = self.rvalue(fs, e[1])
            bf, bt = self.rvalue(fs, e[2])
            return (lambda fr: (af(fr), bf(fr))[1]), bt
        if k == "call":
            return self.callexpr(fs, e)
        if k == "sizeof_t":
            v = sizeof(e[1])
            return (lambda fr: v), ULONG
        if k == "sizeof_e":
            v = sizeof(self.type_of(fs, e[1]))
            return (lambda fr: v), ULONG
        raise CError("expression %r unsupported" % (k,))

    def type_of(self, fs, e):
        """static type of an expression (for sizeof), without decay"""
        if e[0] in ("id", "index", "member", "arrow") or (e[0] == "un" and e[1] == "*"):
            if e[0] == "id" and fs.lookup(e[1]) is None and self.global_type(e[1]) is None:
                return self.rvalue(fs, e)[1]
            return self.lvalue(fs, e)[1]
        return self.rvalue(fs, e)[1]

    def load(self, fs, e):
        lf, t = self.lvalue(fs, e)
        if isinstance(t, Arr):
            el = t.of

            def f(fr):
                b, o = lf(fr)
                return Pointer(b, o, el)
            return f, Ptr(el)

        def g(fr):
            b, o = lf(fr)
            return b[o]
        return g, t

    def unop(self, fs, e):
        op = e[1]
        if op == "&":
            inner = e[2]
            if inner[0] == "un" and inner[1] == "*":
                return self.rvalue(fs, inner[2])
            if inner[0] == "id" and fs.lookup(inner[1]) is None and self.global_type(inner[1]) is None:
                return self.rvalue(fs, inner)  # &function
            lf, t = self.lvalue(fs, inner)

            def f(fr):
                b, o = lf(fr)
                return Pointer(b, o, t)
            return f, Ptr(t)
        af, at = self.rvalue(fs, e[2])
        if op == "!":
            return (lambda fr: 0 if af(fr) else 1), INT
        if isinstance(at, Flt):
            if op == "-":
                return (lambda fr: -af(fr)), at
            return af, at
        rt = promote(at)
        if op == "-":
            return (lambda fr: rt.wrap(-af(fr))), rt
        if op == "+":
            return (lambda fr: rt.wrap(af(fr))), rt
        if op == "~":
            return (lambda fr: rt.wrap(~af(fr))), rt
        raise CError("unary %s" % op)

    def arith(self, op, rt, at, bt):
        """(a, b) -> result for integer binary op in type rt"""
        # FLOAT results are rounded to single after every operation (exact for
        # + - * / of single operands computed in double: 53 >= 2 * 24 + 2)
        w = rt.wrap if isinstance(rt, Int) else (to_f32 if rt.bits == 32 else (lambda v: v))
        if op == "+":
            return lambda a, b: w(a + b)
        if op == "-":
            return lambda a, b: w(a - b)
        if op == "*":
            return lambda a, b: w(a * b)
        if op == "/":
            if isinstance(rt, Flt):
                return lambda a, b: w(a / b)
            return lambda a, b: w(abs(a) // abs(b) * (1 if (a >= 0) == (b >= 0) else -1))
        if op == "%":
            return lambda a, b: w(a - (abs(a) // abs(b) * (1 if (a >= 0) == (b >= 0) else -1)) * b)
        if op == "&":
            return lambda a, b: w(a & b)
        if op == "|":
            return lambda a, b: w(a | b)
        if op == "^":
            return lambda a, b: w(a ^ b)
        raise CError("op %s" % op)

    def binop(self, fs, e):
        op = e[1]
        af, at = self.rvalue(fs, e[2])
        bf, bt = self.rvalue(fs, e[3])
        if op == "&&":
            return (lambda fr: 1 if (af(fr) and bf(fr)) else 0), INT
        if op == "||":
            return (lambda fr: 1 if (af(fr) or bf(fr)) else 0), INT
        if op in ("<<", ">>"):
            rt = promote(at)
            if op == "<<":
                return (lambda fr: rt.wrap(af(fr) << bf(fr))), rt
            if rt.signed:
                return (lambda fr: af(fr) >> bf(fr)), rt
            return (lambda fr: af(fr) >> bf(fr)), rt
        # pointer arithmetic
        if isinstance(at, Ptr) or isinstance(bt, Ptr):
            if op in ("+", "-") and isinstance(at, Ptr) and is_int(bt):
                es = slots(at.to)
                sg = 1 if op == "+" else -1
                return (lambda fr: (lambda p, k: Pointer(p.buf, p.off + sg * k * es, p.ty))(
                    af(fr), bf(fr))), at
            if op == "+" and is_int(at) and isinstance(bt, Ptr):
                es = slots(bt.to)
                return (lambda fr: (lambda k, p: Pointer(p.buf, p.off + k * es, p.ty))(
                    af(fr), bf(fr))), bt
            if op == "-" and isinstance(at, Ptr) and isinstance(bt, Ptr):
                es = slots(at.to)
                return (lambda fr: (af(fr).off - bf(fr).off) // es), LONG
            if op in ("==", "!=", "<", ">", "<=", ">="):
                def key(p):
                    if p is None:
                        return (0, 0)
                    if isinstance(p, Pointer):
                        return (id(p.buf), p.off)
                    if isinstance(p, FuncRef):
                        return (id(p), 0)
                    return (0, p)
                cmpf = {"==": lambda x, y: x == y, "!=": lambda x, y: x != y,
                        "<": lambda x, y: x < y, ">": lambda x, y: x > y,
                        "<=": lambda x, y: x <= y, ">=": lambda x, y: x >= y}[op]
                return (lambda fr: 1 if cmpf(key(af(fr)), key(bf(fr))) else 0), INT
            raise CError("pointer op %s" % op)
        rt = common_type(at, bt)
        ca, cb = self.converter(at, rt), self.converter(bt, rt)
        if op in ("==", "!=", "<", ">", "<=", ">="):
            cmpf = {"==": lambda x, y: x == y, "!=": lambda x, y: x != y,
                    "<": lambda x, y: x < y, ">": lambda x, y: x > y,
                    "<=": lambda x, y: x <= y, ">=": lambda x, y: x >= y}[op]
            if at is rt and bt is rt:
                return (lambda fr: 1 if cmpf(af(fr), bf(fr)) else 0), INT
            return (lambda fr: 1 if cmpf(ca(af(fr)), cb(bf(fr))) else 0), INT
        fn = self.arith(op, rt, at, bt)
        if at is rt and bt is rt:
            return (lambda fr: fn(af(fr), bf(fr))), rt
        return (lambda fr: fn(ca(af(fr)), cb(bf(fr)))), rt

    def assign(self, fs, e):
        op, lhs, rhs = e[1], e[2], e[3]
        lf, lt = self.lvalue(fs, lhs)
        rf, rt_ = self.rvalue(fs, rhs)
        if op == "=":
            if isinstance(lt, Struct):
                def f(fr):
                    b, o = lf(fr)
                    v = copy_obj(rf(fr))
                    b[o] = v
                    return v
                return f, lt
            cv = self.converter(rt_, lt)

            def f(fr):
                v = cv(rf(fr))
                b, o = lf(fr)
                b[o] = v
                return v
            return f, lt
        bop = op[:-1]
        if isinstance(lt, Ptr):
            es = slots(lt.to)
            sg = 1 if bop == "+" else -1

            def f(fr):
                b, o = lf(fr)
                p = b[o]
                v = Pointer(p.buf, p.off + sg * rf(fr) * es, p.ty)
                b[o] = v
                return v
            return f, lt
        if bop in ("<<", ">>"):
            ct = promote(lt)
            if bop == "<<":
                calc = lambda a, b: ct.wrap(a << b)
            else:
                calc = lambda a, b: a >> b
            cr = lambda v: v
        else:
            ct = common_type(lt, rt_)
            calc = self.arith(bop, ct, lt, rt_)
            cr = self.converter(rt_, ct)
        cl = self.converter(lt, ct)
        back = self.converter(ct, lt)

        def f(fr):
            b, o = lf(fr)
            v = back(calc(cl(b[o]), cr(rf(fr))))
            b[o] = v
            return v
        return f, lt

    def incdec(self, fs, e):
        kind, op, inner = e
        lf, lt = self.lvalue(fs, inner)
        d = 1 if op == "++" else -1
        if isinstance(lt, Ptr):
            es = slots(lt.to)

            def step(v):
                return Pointer(v.buf, v.off + d * es, v.ty)
        elif isinstance(lt, Flt):
            step = lambda v: v + d
        else:
            pt = promote(lt)
            step = lambda v: lt.wrap(pt.wrap(v + d))
        if kind == "preinc":
            def f(fr):
                b, o = lf(fr)
                v = step(b[o])
                b[o] = v
                return v
        else:
            def f(fr):
                b, o = lf(fr)
                old = b[o]
                b[o] = step(old)
                return old
        return f, lt

    # ---- calls and builtins ----
    def callexpr(self, fs, e):
        callee, args = e[1], e[2]
        if callee[0] == "id" and fs.lookup(callee[1]) is None:
            name = callee[1]
            b = self.builtin(fs, name, args)
            if b is not None:
                return b
            rn = self.resolve_name(name)
            if rn is not None and self.global_type(name) is None:
                ft = self.func_defs[rn][0]
                argfs = [self.rvalue(fs, a) for a in args]
                convs = [self.converter(at, pt) for (_, at), pt in zip(argfs, ft.params)]
                if len(argfs) != len(ft.params):
                    raise CError("%s: %d args for %d params" % (name, len(args), len(ft.params)))
                fl = [af for af, _ in argfs]
                holder = [None]

                def f(fr):
                    if holder[0] is None:
                        holder[0] = self.compiled.get(rn) or self.compile_func(rn)
                    return holder[0]([cv(a(fr)) for cv, a in zip(convs, fl)])
                return f, ft.ret
        if callee[0] == "id" and fs.lookup(callee[1]) is None and \
                self.global_type(callee[1]) is None and self.resolve_name(callee[1]) is None:
            # no definition: an error only if this call is ever executed
            nm = callee[1]
            ret = self.func_decls[nm].ret if nm in self.func_decls else INT

            def missing(fr):
                raise CError("call to undefined function %s" % nm)
            return missing, ret
        pf, pt = self.rvalue(fs, callee)
        ft = pt.to if isinstance(pt, Ptr) else pt
        if not isinstance(ft, Func):
            raise CError("call of non-function %r" % (pt,))
        argfs = [self.rvalue(fs, a) for a in args]
        convs = [self.converter(at, ptt) for (_, at), ptt in zip(argfs, ft.params)]
        fl = [af for af, _ in argfs]

        def g(fr):
            fn = pf(fr)
            if fn is None:
                raise CError("call through NULL")
            return self.call(fn.name, [cv(a(fr)) for cv, a in zip(convs, fl)])
        return g, ft.ret

    def builtin(self, fs, name, args):
        A = [self.rvalue(fs, a) for a in args] if name not in ("sizeof",) else None
        if name in ("memset",):
            (pf, pt), (vf, _), (nf, _) = A

            def f(fr):
                p, v, n = pf(fr), vf(fr), nf(fr)
                fill_bytes(p, v, n)
                return p
            return f, Ptr(VOID)
        if name in ("memcpy", "memmove"):
            (df, _), (sf, _), (nf, _) = A

            def f(fr):
                d, s, n = df(fr), sf(fr), nf(fr)
                copy_bytes(d, s, n)
                return d
            return f, Ptr(VOID)
        if name in ("abs", "labs", "llabs"):
            (af, at), = A
            rt = INT if name == "abs" else LONG
            return (lambda fr: rt.wrap(abs(af(fr)))), rt
        if name in ("qsort",):
            # glibc qsort on the <= 4-element arrays the reference sorts is an
            # insertion sort (stable); the same here, through the comparator
            (bf, _), (nf, _), _, (cf, _) = A

            def f(fr):
                p, n, cmp = bf(fr), nf(fr), cf(fr)
                cells = p.buf
                for i in range(1, n):
                    k = i
                    while k > 0 and cmp(Pointer(cells, p.off + k - 1, p.ty),
                                        Pointer(cells, p.off + k, p.ty)) > 0:
                        cells[p.off + k - 1], cells[p.off + k] = \
                            cells[p.off + k], cells[p.off + k - 1]
                        k -= 1
                return None
            return f, VOID
        if name in ("assert",):
            return (lambda fr: None), VOID
        if name in ("fprintf", "printf", "fflush"):
            return (lambda fr: 0), INT
        if name in ("__builtin_expect",):  # LIKELY / UNLIKELY (aom_ports/mem.h)
            (af, at), _ = A
            return af, at
        if name in ("__builtin_clz",):
            (af, _), = A
            return (lambda fr: 32 - (af(fr) & 0xFFFFFFFF).bit_length()), INT
        if name in ("__builtin_clzll",):
            (af, _), = A
            return (lambda fr: 64 - (af(fr) & (2 ** 64 - 1)).bit_length()), INT
        if name in ("sqrt",):
            (af, at), = A
            import math
            ca = self.converter(at, DOUBLE)
            return (lambda fr: math.sqrt(ca(af(fr)))), DOUBLE
        if name in ("round",):  # C99 round: half-way cases away from zero, exact
            (af, at), = A
            import math
            ca = self.converter(at, DOUBLE)

            def c_round(x):
                if x != x or math.isinf(x):
                    return x
                a = abs(x)
                fl = math.floor(a)
                return math.copysign(fl + 1.0 if a - fl >= 0.5 else fl, x)
            return (lambda fr: c_round(ca(af(fr)))), DOUBLE
        if name in ("sqrtf",):  # correctly rounded: sqrt in double, then to single
            (af, at), = A
            import math
            ca = self.converter(at, FLOAT)
            return (lambda fr: to_f32(math.sqrt(ca(af(fr))))), FLOAT
        return None

    # ---- statements: fn(frame) -> None | BRK | CONT | RET ----
    def stmt(self, fs, s):
        k = s[0]
        if k == "block":
            fs.scopes.append({})
            parts = [self.stmt(fs, x) for x in s[1]]
            fs.scopes.pop()
            parts = [p for p in parts if p is not None]
            if any(getattr(p, "_case", None) is not None for p in parts):
                raise CError("case label outside switch")

            def f(fr):
                for p in parts:
                    r = p(fr)
                    if r:
                        return r
                return None
            return f
        if k == "decl":
            ops = []
            for name, t, init in s[1]:
                if s[2]["static"] and init is not None and not isinstance(t, Arr):
                    raise CError("static locals unsupported")
                if isinstance(t, Arr) and t.n is None:
                    if init is None:
                        raise CError("incomplete local array")
                    t = Arr(t.of, self.init_count(t, init))
                slot = fs.add(name, t)
                ini = self.store_init(fs, t, init) if init is not None else None
                if s[2]["static"]:
                    # static const table: initialise once, share
                    store = new_storage(t) if isinstance(t, Arr) else [new_obj(t)]
                    if ini is not None:
                        ini(store, 0, [None])
                    ops.append((slot, t, None, store))
                else:
                    ops.append((slot, t, ini, None))

            def f(fr):
                for slot, t, ini, store in ops:
                    if store is not None:
                        fr[slot] = store if isinstance(t, Arr) else store[0]
                        continue
                    if isinstance(t, Arr):
                        fr[slot] = new_storage(t)
                        if ini:
                            ini(fr[slot], 0, fr)
                    else:
                        fr[slot] = new_obj(t)
                        if ini:
                            if isinstance(t, Arr):
                                ini(fr[slot], 0, fr)
                            else:
                                ini(fr, slot, fr)
                return None
            return f
        if k == "expr":
            ef, _ = self.rvalue(fs, s[1])

            def f(fr):
                ef(fr)
                return None
            return f
        if k == "nop":
            return None
        if k == "if":
            cf, _ = self.rvalue(fs, s[1])
            a = self.stmt(fs, s[2]) or (lambda fr: None)
            b = self.stmt(fs, s[3]) if s[3] is not None else None
            if b is None:
                return lambda fr: a(fr) if cf(fr) else None
            return lambda fr: a(fr) if cf(fr) else b(fr)
        if k in ("for", "while", "do"):
            fs.scopes.append({})
            if k == "for":
                init = self.stmt(fs, s[1]) if s[1] is not None else None
                cf = self.rvalue(fs, s[2])[0] if s[2] is not None else (lambda fr: 1)
                step = self.rvalue(fs, s[3])[0] if s[3] is not None else None
                body = self.stmt(fs, s[4]) or (lambda fr: None)
            elif k == "while":
                init, step = None, None
                cf = self.rvalue(fs, s[1])[0]
                body = self.stmt(fs, s[2]) or (lambda fr: None)
            else:
                init, step = None, None
                body = self.stmt(fs, s[1]) or (lambda fr: None)
                cf = self.rvalue(fs, s[2])[0]
            fs.scopes.pop()
            first_check = k != "do"

            def f(fr):
                if init is not None:
                    init(fr)
                chk = first_check
                while True:
                    if chk and not cf(fr):
                        return None
                    chk = True
                    r = body(fr)
                    if r == BRK:
                        return None
                    if r == RET:
                        return RET
                    if step is not None:
                        step(fr)
            return f
        if k == "return":
            if s[1] is None:
                return lambda fr: RET
            ef, et = self.rvalue(fs, s[1])
            cv = self.converter(et, fs.ret)

            def f(fr):
                fr[0] = cv(ef(fr))
                return RET
            return f
        if k == "break":
            return lambda fr: BRK
        if k == "continue":
            return lambda fr: CONT
        if k == "switch":
            cf, ct = self.rvalue(fs, s[1])
            body = s[2]
            items = body[1] if body[0] == "block" else [body]
            fs.scopes.append({})
            labels = {}
            default = None
            parts = []
            for it in self.flatten_cases(items):
                if it[0] == "case":
                    labels[it[1]] = len(parts)
                elif it[0] == "default":
                    default = len(parts)
                else:
                    p = self.stmt(fs, it)
                    parts.append(p or (lambda fr: None))
            fs.scopes.pop()

            def f(fr):
                v = cf(fr)
                start = labels.get(v, default)
                if start is None:
                    return None
                for p in parts[start:]:
                    r = p(fr)
                    if r == BRK:
                        return None
                    if r:
                        return r
                return None
            return f
        raise CError("statement %r unsupported" % (k,))

    def flatten_cases(self, items):
        out = []
        for it in items:
            out.append(it)
        return out

    # ---- host helpers for the fixture generator ----
    def ctype(self, name):
        if name in self.typedefs:
            return self.typedefs[name]
        return Parser(tokenize(name) + [Tok("eof", "<eof>")], self).type_name()

    def buffer(self, tname, values):
        """A Pointer to a fresh flat buffer of element type `tname`."""
        t = self.ctype(tname)
        if isinstance(values, int):
            buf = [new_obj(t) for _ in range(values)] if isinstance(t, Struct) else [0] * values
        else:
            buf = [t.wrap(int(v)) for v in values] if isinstance(t, Int) else list(values)
        return Pointer(buf, 0, t)

    def struct_obj(self, tname):
        t = self.ctype(tname)
        buf = [new_obj(t)]
        return Pointer(buf, 0, t)

    def tagged(self, p):
        """CONVERT_TO_BYTEPTR(p) (aom_ports/mem.h:80): the uint8_t* a highbd
        caller passes for a uint16_t buffer."""
        return Pointer(None, self.addr.to_int(p) >> 1, UCHAR)

    def global_value(self, name):
        cell, off, t = self.global_cell(name)
        if isinstance(t, Arr):
            return cell
        return cell[0]


def fill_bytes(p, v, n):
    t = p.ty
    el = scalar_of(t) if not isinstance(t, Void) else UCHAR
    if isinstance(el, Struct):
        sz = sizeof(el)
        cnt = n // sz
        if v != 0:
            raise CError("memset of structs to nonzero")
        for k in range(cnt):
            p.buf[p.off + k] = new_obj(el)
        return
    es = sizeof(el)
    if n % es:
        raise CError("memset of a partial element")
    cnt = n // es
    if v != 0 and es != 1:
        raise CError("memset of multi-byte elements to nonzero")
    val = el.wrap(v) if isinstance(el, Int) else (0.0 if v == 0 else None)
    if isinstance(t, Struct):
        raise CError("memset of a struct")
    p.buf[p.off:p.off + cnt] = [val] * cnt


def copy_bytes(d, s, n):
    el = scalar_of(d.ty)
    es = sizeof(el)
    if sizeof(scalar_of(s.ty)) != es:
        raise CError("memcpy between different element sizes")
    cnt = n // es
    d.buf[d.off:d.off + cnt] = [copy_obj(x) for x in s.buf[s.off:s.off + cnt]]


# =============================================================================
# configuration: the reference's CMake defaults
# =============================================================================
def reference_defines(root):
    """CONFIG_* defaults from build/cmake/aom_config_defaults.cmake (the
    reference's own file), plus what its generated config/aom_config.h
    states for a generic (no SIMD) x86-64 gcc build: HAVE_* 0, INLINE
    inline, and the compiler macros the headers test."""
    d = {}
    with open(os.path.join(root, "build/cmake/aom_config_defaults.cmake")) as f:
        txt = f.read()
    for m in re.finditer(r"set_aom_config_var\(\s*(\w+)\s+(\w+)", txt):
        name, val = m.group(1), m.group(2)
        if re.fullmatch(r"-?\d+", val):
            d[name] = int(val)
    for k in list(d):
        if k.startswith("HAVE_") or k.startswith("AOM_ARCH_") or k.startswith("ARCH_"):
            d[k] = 0
    d.update({"INLINE": "inline", "__GNUC__": 11, "__GNUC_MINOR__": 4, "__x86_64__": 1,
              "__STDC_VERSION__": 201112, "NDEBUG": 1, "INT16_MIN": "(-32768)",
              "INT16_MAX": "32767", "INT32_MIN": "(-2147483647-1)", "INT32_MAX": "2147483647",
              "INT64_MAX": "9223372036854775807L", "INT64_MIN": "(-9223372036854775807L-1)",
              "UINT32_MAX": "4294967295U", "UINT16_MAX": "65535", "INT8_MAX": "127",
              "INT8_MIN": "(-128)", "UINT8_MAX": "255", "UINT64_MAX": "18446744073709551615UL",
              "INT_MAX": "2147483647", "INT_MIN": "(-2147483647-1)", "NULL": "((void*)0)",
              "CHAR_BIT": "8", "UINT_MAX": "4294967295U", "bool": "_Bool", "true": "1",
              "false": "0"})
    return d
