"""Rego value model for the oracle (test infrastructure only).

Restates the OPA v0.21 value semantics the audit path depends on:

* numbers keep their JSON/literal text; comparison is int64 when both texts
  parse as int64, else big.Float at 64-bit mantissa, round-half-even
  (``vendor/github.com/open-policy-agent/opa/ast/compare.go:87-108``);
  arithmetic is big.Float Mul/Add/... then ``Text('g', -1)``
  (``topdown/arithmetic.go:43-45``, ``topdown/builtins/builtins.go:161-172``);
* sets and objects keep insertion order (``ast/term.go:1167-1170, 1522-1526``);
* ``Term.String()`` printing (``ast/term.go:506-507, 555-557, 647-649, 700-702,
  1112-1118, 1197-1206, 1807-1813``) and Go ``fmt.Sprintf`` conversion in
  ``sprintf`` (``topdown/strings.go:340-371``);
* Go ``encoding/json`` marshalling of result bindings (sorted map keys, HTML
  escaping) used by ``drivers/local/local.go:341-352``.
"""
from __future__ import annotations

import json
import math
from fractions import Fraction

# --------------------------------------------------------------------------
# scalar singletons
# --------------------------------------------------------------------------


class _Null:
    __slots__ = ()

    def __repr__(self):
        return "NULL"

    def __hash__(self):
        return hash("__rego_null__")

    def __eq__(self, o):
        return o is self


NULL = _Null()


class RegoError(Exception):
    """A builtin/evaluation error: aborts the whole query (topdown/builtins.go:145-164)."""


class ConflictError(RegoError):
    pass


# --------------------------------------------------------------------------
# big.Float emulation at 64-bit mantissa, ToNearestEven
# --------------------------------------------------------------------------
PREC = 64
_TWO64 = 1 << 64
_TWO63 = 1 << 63


def bf_round(fr: Fraction):
    """Round an exact rational to a 64-bit-mantissa binary float.

    Returns (neg, mant, exp) with value = mant * 2**exp, mant in [2^63, 2^64),
    or None for zero.  Mirrors math/big Float.SetString / Mul rounding at
    prec 64, mode ToNearestEven.
    """
    if fr == 0:
        return None
    neg = fr < 0
    fr = -fr if neg else fr
    n, d = fr.numerator, fr.denominator
    e = n.bit_length() - d.bit_length() - PREC
    while True:
        if e >= 0:
            den = d << e
            q, r = divmod(n, den)
        else:
            den = d
            q, r = divmod(n << (-e), d)
        if q >= _TWO64:
            e += 1
            continue
        if q < _TWO63:
            e -= 1
            continue
        break
    if 2 * r > den or (2 * r == den and (q & 1)):
        q += 1
        if q == _TWO64:
            q >>= 1
            e += 1
    return (neg, q, e)


def bf_to_fraction(bf) -> Fraction:
    if bf is None:
        return Fraction(0)
    neg, m, e = bf
    v = Fraction(m) * (Fraction(2) ** e)
    return -v if neg else v


def _parse_decimal_text(text: str) -> Fraction:
    """Exact value of a Go big.Float-parsable decimal number text."""
    t = text.strip()
    if t == "" or any(c in t for c in "_xXpP") or t.lower().lstrip("+-") in ("inf", "infinity", "nan"):
        raise ValueError(text)
    return Fraction(t)


def _int64_text(text: str):
    """json.Number(text).Int64() == strconv.ParseInt(text, 10, 64)."""
    t = text
    if not t:
        return None
    body = t[1:] if t[0] in "+-" else t
    if not body or not body.isdigit() or not body.isascii():
        return None
    v = int(t)
    if v < -(1 << 63) or v > (1 << 63) - 1:
        return None
    return v


def _decimal_digits(fr: Fraction):
    """Exact decimal expansion of a dyadic rational: (digits, dp) so that
    value = 0.digits * 10**dp (Go math/big decimal), digits without
    leading/trailing zeros."""
    n, d = fr.numerator, fr.denominator
    assert n > 0
    # d is a power of two
    k = d.bit_length() - 1
    assert d == 1 << k
    digits_int = n * (5 ** k)  # value = digits_int * 10**-k
    s = str(digits_int)
    dp = len(s) - k
    s = s.rstrip("0")
    return s, dp


def _round_digits(s: str, dp: int, n: int, mode: str):
    """Round decimal (s, dp) to n digits; mode in {'near','down','up'}."""
    if n < 0 or n >= len(s):
        return s, dp
    if mode == "down":
        s2 = s[:n]
    else:
        up = True
        if mode == "near":
            c = s[n]
            if c == "5" and n + 1 == len(s):
                up = n > 0 and (int(s[n - 1]) & 1) == 1
            else:
                up = c >= "5"
        if not up:
            s2 = s[:n]
        else:
            # round up: increment the n-digit prefix
            digs = list(s[:n])
            i = n - 1
            while i >= 0 and digs[i] == "9":
                i -= 1
            if i < 0:
                s2 = "1"
                dp += 1
            else:
                digs[i] = chr(ord(digs[i]) + 1)
                s2 = "".join(digs[: i + 1])
    s2 = s2.rstrip("0")
    return s2, dp


def bf_text_g_shortest(bf) -> str:
    """math/big Float.Text('g', -1) at prec 64 (ftoa.go roundShortest + %g)."""
    if bf is None:
        return "0"
    neg, m, e = bf
    x = Fraction(m) * (Fraction(2) ** e)
    s, dp = _decimal_digits(x)
    # roundShortest: mant with prec+1 bits, lsb = 1/2 ulp
    mant = m << 1
    exp = e - 1
    inclusive = (mant & 2) == 0
    lower = Fraction(mant - 1) * (Fraction(2) ** exp)
    upper = Fraction(mant + 1) * (Fraction(2) ** exp)
    ls, ldp = _decimal_digits(lower)
    us, udp = _decimal_digits(upper)

    def at(ds, ddp, i):
        # digit i of d's mantissa when aligned at d's dp (Go decimal.at with same exp)
        # Go compares lower.at(i)/upper.at(i) after all three share the same
        # decimal exponent; they do here because lower/upper straddle x closely.
        return ds[i] if 0 <= i < len(ds) else "0"

    # Align lower/upper to x's decimal point (pad with leading zeros if needed)
    def align(ds, ddp):
        if ddp < dp:
            return "0" * (dp - ddp) + ds
        if ddp > dp:
            # upper may have carried into a new digit; shift
            return ds  # Go: exponents differ -> digits differ at i=0, handled below
        return ds

    la = align(ls, ldp)
    ua = align(us, udp)
    if udp > dp:
        ua = "@" + ua  # forces u != m at the first digit
    for i in range(len(s)):
        mch = s[i]
        lch = at(la, dp, i)
        uch = ua[i] if i < len(ua) else "0"
        okdown = lch != mch or (inclusive and i + 1 == len(la))
        if uch == "@":
            okup = True
        else:
            okup = mch != uch and (inclusive or int(mch) + 1 < int(uch) or i + 1 < len(ua))
        if okdown and okup:
            s, dp = _round_digits(s, dp, i + 1, "near")
            break
        if okdown:
            s, dp = _round_digits(s, dp, i + 1, "down")
            break
        if okup:
            s, dp = _round_digits(s, dp, i + 1, "up")
            break
    out = _fmt_g_shortest(s, dp)
    return ("-" + out) if neg else out


def _fmt_g_shortest(s: str, dp: int) -> str:
    prec = len(s)
    eprec = 6
    exp = dp - 1
    if exp < -4 or exp >= eprec:
        # fmtE with prec-1 fractional digits
        buf = s[0]
        if prec - 1 > 0:
            buf += "." + s[1:prec]
        buf += "e"
        if exp < 0:
            buf += "-"
            exp = -exp
        else:
            buf += "+"
        if exp < 10:
            buf += "0"
        buf += str(exp)
        return buf
    # fmtF with max(prec-dp, 0) fractional digits
    if prec > dp:
        pass
    fr = max(prec - dp, 0)
    if dp > 0:
        ip = s[:dp] + "0" * max(0, dp - len(s))
    else:
        ip = "0"
    if fr > 0:
        frac = ""
        for i in range(1, fr + 1):
            j = dp + i - 1
            frac += s[j] if 0 <= j < len(s) else "0"
        return ip + "." + frac
    return ip


class Num:
    """A Rego number (ast.Number): its text plus an exact comparison key."""

    __slots__ = ("text", "_i", "_bf", "_hash")

    def __init__(self, text: str):
        self.text = text
        self._i = _int64_text(text)
        self._bf = "unset"
        self._hash = None

    @classmethod
    def from_int(cls, v: int) -> "Num":
        return cls(str(v))

    @classmethod
    def from_bf(cls, bf) -> "Num":
        return cls(bf_text_g_shortest(bf))

    @property
    def int64(self):
        return self._i

    @property
    def bf(self):
        if self._bf == "unset":
            try:
                self._bf = bf_round(_parse_decimal_text(self.text))
            except (ValueError, ZeroDivisionError):
                raise RegoError("illegal value")
        return self._bf

    def cmp(self, other: "Num") -> int:
        if self._i is not None and other._i is not None:
            return (self._i > other._i) - (self._i < other._i)
        a = bf_to_fraction(self.bf)
        b = bf_to_fraction(other.bf)
        return (a > b) - (a < b)

    def __eq__(self, o):
        return isinstance(o, Num) and self.cmp(o) == 0

    def __hash__(self):
        if self._hash is None:
            if self._i is not None:
                self._hash = hash(("num", Fraction(self._i)))
            else:
                try:
                    self._hash = hash(("num", bf_to_fraction(self.bf)))
                except RegoError:
                    self._hash = hash(("numtext", self.text))
        return self._hash

    def __repr__(self):
        return "Num(%s)" % self.text


class Arr(tuple):
    """Rego array (ordered, hashable)."""

    def __repr__(self):
        return "Arr(%s)" % (list(self),)


class Obj:
    """Rego object: insertion-ordered, hashable by content."""

    __slots__ = ("_d", "_hash")

    def __init__(self, items=()):
        d = {}
        for k, v in items:
            d[k] = v
        self._d = d
        self._hash = None

    def get(self, k, default=None):
        return self._d.get(k, default)

    def __contains__(self, k):
        return k in self._d

    def keys(self):
        return self._d.keys()

    def items(self):
        return self._d.items()

    def values(self):
        return self._d.values()

    def __len__(self):
        return len(self._d)

    def __eq__(self, o):
        if not isinstance(o, Obj) or len(o) != len(self):
            return False
        for k, v in self._d.items():
            if k not in o._d or not rego_equal(o._d[k], v):
                return False
        return True

    def __hash__(self):
        if self._hash is None:
            self._hash = hash(("obj", frozenset((k, _h(v)) for k, v in self._d.items())))
        return self._hash

    def with_item(self, k, v) -> "Obj":
        o = Obj()
        o._d = dict(self._d)
        o._d[k] = v
        return o

    def __repr__(self):
        return "Obj(%s)" % (list(self._d.items()),)


class RSet:
    """Rego set: insertion-ordered, dedup by Rego equality."""

    __slots__ = ("_d", "_hash")

    def __init__(self, items=()):
        d = {}
        for x in items:
            if x not in d:
                d[x] = None
        self._d = d
        self._hash = None

    def __iter__(self):
        return iter(self._d)

    def __len__(self):
        return len(self._d)

    def __contains__(self, x):
        return x in self._d

    def add(self, x):
        if x not in self._d:
            self._d[x] = None
            self._hash = None

    def __eq__(self, o):
        return isinstance(o, RSet) and len(o) == len(self) and all(x in o._d for x in self._d)

    def __hash__(self):
        if self._hash is None:
            self._hash = hash(("set", frozenset(_h(x) for x in self._d)))
        return self._hash

    def __repr__(self):
        return "RSet(%s)" % (list(self._d),)


def _h(v):
    return hash(v) if not isinstance(v, bool) else hash(("bool", v))


# Python's True == 1 would collide with Num-like keys in dicts; values are
# always wrapped so ints never appear, but bools are still ints: use a
# distinct wrapper key for hashing via _BoolKey in sets/dicts.
def type_order(v) -> int:
    """ast.sortOrder: null < boolean < number < string < ... < array < object < set."""
    if v is NULL:
        return 1
    if isinstance(v, bool):
        return 2
    if isinstance(v, Num):
        return 3
    if isinstance(v, str):
        return 4
    if isinstance(v, Arr):
        return 7
    if isinstance(v, Obj):
        return 8
    if isinstance(v, RSet):
        return 9
    raise TypeError("not a rego value: %r" % (v,))


def rego_compare(a, b) -> int:
    """ast.Compare (compare.go:39-226)."""
    ta, tb = type_order(a), type_order(b)
    if ta != tb:
        return -1 if ta < tb else 1
    if ta == 1:
        return 0
    if ta == 2:
        return (a > b) - (a < b)
    if ta == 3:
        return a.cmp(b)
    if ta == 4:
        ab, bb = a.encode("utf-8", "surrogateescape"), b.encode("utf-8", "surrogateescape")
        return (ab > bb) - (ab < bb)
    if ta == 7:
        for x, y in zip(a, b):
            c = rego_compare(x, y)
            if c:
                return c
        return (len(a) > len(b)) - (len(a) < len(b))
    if ta == 8:
        # sorted (key,value) pairs, then length
        ka = sorted(a.keys(), key=_cmp_key)
        kb = sorted(b.keys(), key=_cmp_key)
        for x, y in zip(ka, kb):
            c = rego_compare(x, y)
            if c:
                return c
            c = rego_compare(a.get(x), b.get(y))
            if c:
                return c
        return (len(ka) > len(kb)) - (len(ka) < len(kb))
    if ta == 9:
        sa = sorted(a, key=_cmp_key)
        sb = sorted(b, key=_cmp_key)
        for x, y in zip(sa, sb):
            c = rego_compare(x, y)
            if c:
                return c
        return (len(sa) > len(sb)) - (len(sa) < len(sb))
    raise TypeError


class _CmpKey:
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v

    def __lt__(self, o):
        return rego_compare(self.v, o.v) < 0


def _cmp_key(v):
    return _CmpKey(v)


def rego_equal(a, b) -> bool:
    if isinstance(a, bool) or isinstance(b, bool):
        return isinstance(a, bool) and isinstance(b, bool) and a == b
    try:
        return rego_compare(a, b) == 0
    except TypeError:
        return False


def sort_values(vals):
    return sorted(vals, key=_cmp_key)


# --------------------------------------------------------------------------
# JSON <-> value
# --------------------------------------------------------------------------


def from_json_text(text: str):
    """util.RoundTrip + ast.InterfaceToValue: numbers keep their text."""
    raw = json.loads(text, parse_float=lambda s: ("__num__", s), parse_int=lambda s: ("__num__", s),
                     object_pairs_hook=lambda pairs: ("__obj__", pairs))
    return from_py(raw)


def from_py(x):
    if isinstance(x, tuple) and len(x) == 2 and x[0] == "__num__":
        return Num(x[1])
    if isinstance(x, tuple) and len(x) == 2 and x[0] == "__obj__":
        return Obj((k, from_py(v)) for k, v in x[1])
    if x is None:
        return NULL
    if isinstance(x, bool):
        return x
    if isinstance(x, int):
        return Num(str(x))
    if isinstance(x, float):
        return Num(_go_float_json(x))
    if isinstance(x, str):
        return x
    if isinstance(x, dict):
        return Obj((k, from_py(v)) for k, v in x.items())
    if isinstance(x, (list, tuple)):
        return Arr(from_py(v) for v in x)
    if isinstance(x, (Num, Obj, Arr, RSet, _Null)):
        return x
    raise TypeError("cannot convert %r" % (x,))


def _go_float_json(f: float) -> str:
    # encoding/json float64 formatting (ES6-like)
    if f == int(f) and abs(f) < 1e21:
        return str(int(f))
    r = repr(f)
    return r


def to_py(v):
    """Rego value -> plain Python (sets -> lists, numbers -> int/float/str-text)."""
    if v is NULL:
        return None
    if isinstance(v, bool) or isinstance(v, str):
        return v
    if isinstance(v, Num):
        if v.int64 is not None:
            return v.int64
        return float(v.text)
    if isinstance(v, Arr):
        return [to_py(x) for x in v]
    if isinstance(v, RSet):
        return [to_py(x) for x in v]
    if isinstance(v, Obj):
        return {_key_str(k): to_py(x) for k, x in v.items()}
    raise TypeError(v)


def _key_str(k):
    if isinstance(k, str):
        return k
    return term_string(k)


def go_json_marshal(v) -> str:
    """encoding/json.Marshal of ast.JSON(v): map keys sorted, HTML-escaped strings."""
    if v is NULL:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, Num):
        return v.text
    if isinstance(v, str):
        return go_json_string(v)
    if isinstance(v, (Arr, RSet)):
        return "[" + ",".join(go_json_marshal(x) for x in v) + "]"
    if isinstance(v, Obj):
        items = sorted(((_key_str(k), x) for k, x in v.items()), key=lambda kv: kv[0].encode("utf-8", "surrogateescape"))
        return "{" + ",".join(go_json_string(k) + ":" + go_json_marshal(x) for k, x in items) + "}"
    raise TypeError(v)


_HEX = "0123456789abcdef"


def go_json_string(s: str) -> str:
    out = ['"']
    for ch in s:
        c = ord(ch)
        if 0xDC80 <= c <= 0xDCFF:  # surrogate-escaped invalid byte
            out.append("\\ufffd")
        elif ch == '"':
            out.append('\\"')
        elif ch == "\\":
            out.append("\\\\")
        elif ch == "\n":
            out.append("\\n")
        elif ch == "\r":
            out.append("\\r")
        elif ch == "\t":
            out.append("\\t")
        elif c < 0x20 or ch in "<>&" or c in (0x2028, 0x2029):
            out.append("\\u%04x" % c)
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


# --------------------------------------------------------------------------
# printing
# --------------------------------------------------------------------------


def go_quote(s: str) -> str:
    """strconv.Quote (Go 1.15): escape non-printable runes; invalid UTF-8 -> \\xHH."""
    out = ['"']
    for ch in s:
        c = ord(ch)
        if 0xDC80 <= c <= 0xDCFF:
            out.append("\\x%02x" % (c - 0xDC00))
            continue
        if ch == '"' or ch == "\\":
            out.append("\\" + ch)
            continue
        if ch.isprintable():
            out.append(ch)
            continue
        m = {"\a": "\\a", "\b": "\\b", "\f": "\\f", "\n": "\\n", "\r": "\\r", "\t": "\\t", "\v": "\\v"}
        if ch in m:
            out.append(m[ch])
        elif c < 0x20 or c == 0x7F:
            out.append("\\x%02x" % c)
        elif c < 0x10000:
            out.append("\\u%04x" % c)
        else:
            out.append("\\U%08x" % c)
    out.append('"')
    return "".join(out)


def term_string(v) -> str:
    """ast.Term.String() / Value.String()."""
    if v is NULL:
        return "null"
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, Num):
        return v.text
    if isinstance(v, str):
        return go_quote(v)
    if isinstance(v, Arr):
        return "[" + ", ".join(term_string(x) for x in v) + "]"
    if isinstance(v, RSet):
        if len(v) == 0:
            return "set()"
        return "{" + ", ".join(term_string(x) for x in v) + "}"
    if isinstance(v, Obj):
        return "{" + ", ".join(term_string(k) + ": " + term_string(x) for k, x in v.items()) + "}"
    raise TypeError(v)


def _go_float_v(f: float) -> str:
    """fmt %v of a float64: strconv 'g' shortest, %e when exp < -4 || exp >= 6
    (strconv/ftoa.go: shortest => eprec = 6)."""
    if math.isinf(f):
        return "+Inf" if f > 0 else "-Inf"
    if math.isnan(f):
        return "NaN"
    if f == 0:
        return "-0" if math.copysign(1, f) < 0 else "0"
    r = repr(abs(f))
    # extract digits and exponent from python shortest repr
    if "e" in r:
        mant, ex = r.split("e")
        ex = int(ex)
    else:
        mant, ex = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    lead = len(ip + fp) - len((ip + fp).lstrip("0"))
    dp = len(ip) + ex - lead
    digits = digits.rstrip("0") or "0"
    exp = dp - 1
    if exp < -4 or exp >= 6:
        buf = digits[0]
        if len(digits) > 1:
            buf += "." + digits[1:]
        buf += "e" + ("-" if exp < 0 else "+") + ("0" if abs(exp) < 10 else "") + str(abs(exp))
    else:
        if dp <= 0:
            buf = "0." + "0" * (-dp) + digits
        elif dp >= len(digits):
            buf = digits + "0" * (dp - len(digits))
        else:
            buf = digits[:dp] + "." + digits[dp:]
    return ("-" + buf) if f < 0 else buf


def sprintf_arg(v):
    """strings.go:355-367 conversion of one sprintf argument to a Go value."""
    if isinstance(v, Num):
        if v.int64 is not None:
            return ("int", v.int64)
        try:
            f = float(_parse_decimal_text(v.text))
            if math.isinf(f):
                raise OverflowError
            return ("float64", f)
        except (ValueError, OverflowError):
            return ("string", v.text)
    if isinstance(v, str):
        return ("string", v)
    return ("string", term_string(v))


def go_sprintf(fmt: str, args) -> str:
    """Go fmt.Sprintf for the verbs the templates use (%v %s %d %q %%)."""
    conv = [sprintf_arg(a) for a in args]
    out = []
    i = 0
    argi = 0
    n = len(fmt)
    while i < n:
        ch = fmt[i]
        if ch != "%":
            out.append(ch)
            i += 1
            continue
        i += 1
        if i >= n:
            out.append("%!(NOVERB)")
            break
        # flags / width are not used by the templates; support plain verbs
        verb = fmt[i]
        i += 1
        if verb == "%":
            out.append("%")
            continue
        if argi >= len(conv):
            out.append("%!" + verb + "(MISSING)")
            continue
        kind, val = conv[argi]
        argi += 1
        out.append(_fmt_one(verb, kind, val))
    if argi < len(conv):
        extra = ", ".join(_go_type(k) + "=" + _fmt_one("v", k, v) for k, v in conv[argi:])
        out.append("%!(EXTRA " + extra + ")")
    return "".join(out)


def _go_type(k):
    return {"int": "int", "float64": "float64", "string": "string"}[k]


def _fmt_one(verb, kind, val):
    if kind == "int":
        if verb in "vd":
            return str(val)
        if verb == "s":
            return "%!s(int=" + str(val) + ")"
        if verb == "q":
            return "'" + chr(val) + "'" if 0 <= val < 0x110000 else "%!q(int=" + str(val) + ")"
    if kind == "float64":
        if verb == "v" or verb == "g":
            return _go_float_v(val) if verb == "v" else _go_float_v(val)
        if verb == "s":
            return "%!s(float64=" + _go_float_v(val) + ")"
        if verb == "d":
            return "%!d(float64=" + _go_float_v(val) + ")"
    if kind == "string":
        if verb in "vs":
            return val
        if verb == "q":
            return go_quote(val)
        if verb == "d":
            return "%!d(string=" + val + ")"
    raise NotImplementedError("sprintf verb %%%s for %s" % (verb, kind))
