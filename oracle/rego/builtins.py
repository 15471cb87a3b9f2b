"""OPA v0.21 builtins used by the audit path — oracle restatement (test infra only).

File:line anchors (``vendor/github.com/open-policy-agent/opa/topdown``):
count/any/all ``aggregates.go:14-203``; arithmetic ``arithmetic.go:43-119``;
casts ``casts.go:14-33``; strings ``strings.go:48-371``; regex ``regex.go:21-34``;
type checks ``type.go``; comparison ``compare.go`` (ast.Compare).
"""
from __future__ import annotations

from fractions import Fraction

from . import goregex
from .values import (NULL, Arr, Num, Obj, RegoError, RSet, bf_round, bf_to_fraction, go_sprintf, rego_compare,
                     rego_equal, sort_values, term_string, type_order)


def _type_name(v):
    if v is NULL:
        return "null"
    if isinstance(v, bool):
        return "boolean"
    if isinstance(v, Num):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, Arr):
        return "array"
    if isinstance(v, Obj):
        return "object"
    if isinstance(v, RSet):
        return "set"
    return "?"


def _err(pos, v, *want):
    raise RegoError("operand %d must be %s but got %s" % (pos, " or ".join(want), _type_name(v)))


def _str(v, pos):
    if not isinstance(v, str):
        _err(pos, v, "string")
    return v


def _num(v, pos):
    if not isinstance(v, Num):
        _err(pos, v, "number")
    return v


def _int(v, pos):
    n = _num(v, pos)
    fr = bf_to_fraction(n.bf)
    if fr.denominator != 1:
        raise RegoError("operand %d must be integer number but got floating-point number" % pos)
    return int(fr)


def _blen(s: str) -> int:
    return len(s.encode("utf-8", "surrogateescape"))


def _b(s: str) -> bytes:
    return s.encode("utf-8", "surrogateescape")


def _s(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


# ---------------------------------------------------------------- aggregates
def count(a):
    if isinstance(a, (Arr, RSet, Obj)):
        return Num(str(len(a)))
    if isinstance(a, str):
        return Num(str(_blen(a)))
    _err(1, a, "array", "object", "set")


def any_(a):
    if isinstance(a, RSet):
        return True in a
    if isinstance(a, Arr):
        return any(x is True for x in a)
    _err(1, a, "array", "set")


def all_(a):
    if isinstance(a, RSet):
        return all(x is True for x in a)
    if isinstance(a, Arr):
        return all(x is True for x in a)
    _err(1, a, "array", "set")


def _arith(fn):
    def f(a, b):
        _num(a, 1)
        _num(b, 2)
        return Num.from_bf(bf_round(fn(bf_to_fraction(a.bf), bf_to_fraction(b.bf))))
    return f


def plus(a, b):
    return _arith(lambda x, y: x + y)(a, b)


def mul(a, b):
    return _arith(lambda x, y: x * y)(a, b)


def minus(a, b):
    if isinstance(a, Num) and isinstance(b, Num):
        return _arith(lambda x, y: x - y)(a, b)
    if isinstance(a, RSet) and isinstance(b, RSet):
        return RSet(x for x in a if x not in b)
    if not isinstance(a, (Num, RSet)):
        _err(1, a, "number", "set")
    _err(2, b, "number", "set")


def div(a, b):
    _num(a, 1)
    _num(b, 2)
    fb = bf_to_fraction(b.bf)
    if fb == 0:
        raise RegoError("divide by zero")
    # big.Float Quo at prec 64 of the (rounded) operands
    return Num.from_bf(bf_round(bf_to_fraction(a.bf) / fb))


def rem(a, b):
    x = _int(a, 1)
    y = _int(b, 2)
    if y == 0:
        raise RegoError("modulo by zero")
    r = abs(x) % abs(y)
    return Num(str(-r if x < 0 else r))


def set_or(a, b):
    if not isinstance(a, RSet):
        _err(1, a, "set")
    if not isinstance(b, RSet):
        _err(2, b, "set")
    out = RSet(a)
    for x in b:
        out.add(x)
    return out


def set_and(a, b):
    if not isinstance(a, RSet):
        _err(1, a, "set")
    if not isinstance(b, RSet):
        _err(2, b, "set")
    return RSet(x for x in a if x in b)


# ---------------------------------------------------------------- comparison
def equal(a, b):
    return rego_equal(a, b)


def neq(a, b):
    return not rego_equal(a, b)


def lt(a, b):
    return rego_compare(a, b) < 0


def lte(a, b):
    return rego_compare(a, b) <= 0


def gt(a, b):
    return rego_compare(a, b) > 0


def gte(a, b):
    return rego_compare(a, b) >= 0


# ---------------------------------------------------------------- strings
def startswith(a, b):
    return _b(_str(a, 1)).startswith(_b(_str(b, 2)))


def endswith(a, b):
    return _b(_str(a, 1)).endswith(_b(_str(b, 2)))


def contains(a, b):
    return _b(_str(b, 2)) in _b(_str(a, 1))


def replace(s, old, new):
    return _s(_b(_str(s, 1)).replace(_b(_str(old, 2)), _b(_str(new, 3))))


def substring(s, start, length):
    base = _b(_str(s, 1))
    st = _int(start, 2)
    if st >= len(base):
        return ""
    if st < 0:
        raise RegoError("negative offset")
    ln = _int(length, 3)
    if ln < 0:
        return _s(base[st:])
    return _s(base[st:min(len(base), st + ln)])


def split(s, d):
    return Arr(_s(x) for x in _go_split(_b(_str(s, 1)), _b(_str(d, 2))))


def _go_split(s: bytes, sep: bytes):
    if sep == b"":
        # strings.Split with empty sep: split into UTF-8 sequences
        return [ch.encode("utf-8", "surrogateescape") for ch in _s(s)]
    return s.split(sep)


def concat(d, arr):
    _str(d, 1)
    if isinstance(arr, (Arr, RSet)):
        parts = []
        for x in arr:
            if not isinstance(x, str):
                raise RegoError("operand 2 must be array of strings")
            parts.append(x)
        return d.join(parts)
    _err(2, arr, "set", "array")


def trim(s, cutset):
    s = _str(s, 1)
    c = set(_str(cutset, 2))
    i, j = 0, len(s)
    while i < j and s[i] in c:
        i += 1
    while j > i and s[j - 1] in c:
        j -= 1
    return s[i:j]


def trim_prefix(s, p):
    s = _str(s, 1)
    p = _str(p, 2)
    return s[len(p):] if s.startswith(p) else s


def trim_suffix(s, p):
    s = _str(s, 1)
    p = _str(p, 2)
    return s[:-len(p)] if p and s.endswith(p) else s


def lower(s):
    return _str(s, 1).lower()


def upper(s):
    return _str(s, 1).upper()


def indexof(s, sub):
    b = _b(_str(s, 1)).find(_b(_str(sub, 2)))
    return Num(str(b))


def sprintf(fmt, arr):
    _str(fmt, 1)
    if not isinstance(arr, Arr):
        _err(2, arr, "array")
    return go_sprintf(fmt, list(arr))


def re_match(pattern, value):
    return goregex.re_match(_str(pattern, 1), _str(value, 2))


# ---------------------------------------------------------------- casts/types
def to_number(a):
    if a is NULL:
        return Num("0")
    if isinstance(a, bool):
        return Num("1" if a else "0")
    if isinstance(a, Num):
        return a
    if isinstance(a, str):
        if not _go_parse_float_ok(a):
            raise RegoError('strconv.ParseFloat: parsing %s: invalid syntax' % term_string(a))
        return Num(a)
    _err(1, a, "null", "boolean", "number", "string")


def _go_parse_float_ok(s: str) -> bool:
    """strconv.ParseFloat(s, 64) accepts (decimal forms; inf/nan/hex refused
    conservatively as NotImplemented)."""
    import re as _re
    if _re.fullmatch(r"[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?", s):
        return True
    low = s.lower().lstrip("+-")
    if low in ("inf", "infinity", "nan") or low.startswith("0x") or "_" in s:
        raise NotImplementedError("ParseFloat special form %r" % s)
    return False


def is_number(a):
    return isinstance(a, Num)


def is_string(a):
    return isinstance(a, str)


def is_boolean(a):
    return isinstance(a, bool)


def is_array(a):
    return isinstance(a, Arr)


def is_set(a):
    return isinstance(a, RSet)


def is_object(a):
    return isinstance(a, Obj)


def is_null(a):
    return a is NULL


def type_name(a):
    return _type_name(a)


def sort(a):
    if isinstance(a, (Arr, RSet)):
        return Arr(sort_values(list(a)))
    _err(1, a, "array", "set")


def array_concat(a, b):
    """topdown/array.go builtinArrayConcat: both operands arrays."""
    if not isinstance(a, Arr):
        _err(1, a, "array")
    if not isinstance(b, Arr):
        _err(2, b, "array")
    return Arr(list(a) + list(b))


def abs_(a):
    n = _num(a, 1)
    return Num.from_bf(bf_round(abs(bf_to_fraction(n.bf))))


def max_(a):
    if isinstance(a, (Arr, RSet)):
        vals = list(a)
        if not vals:
            return None
        m = vals[0]
        for x in vals[1:]:
            if rego_compare(x, m) > 0:
                m = x
        return m
    _err(1, a, "set", "array")


def min_(a):
    if isinstance(a, (Arr, RSet)):
        vals = list(a)
        if not vals:
            return None
        m = vals[0]
        for x in vals[1:]:
            if rego_compare(x, m) < 0:
                m = x
        return m
    _err(1, a, "set", "array")


def sum_(a):
    if isinstance(a, (Arr, RSet)):
        acc = Fraction(0)
        for x in a:
            if not isinstance(x, Num):
                raise RegoError("operand 1 must be array/set of numbers")
            acc = bf_to_fraction(bf_round(acc + bf_to_fraction(x.bf)))
        return Num.from_bf(bf_round(acc))
    _err(1, a, "set", "array")


BUILTINS = {
    "count": count, "any": any_, "all": all_, "sum": sum_, "max": max_, "min": min_,
    "plus": plus, "minus": minus, "mul": mul, "div": div, "rem": rem, "abs": abs_,
    "or": set_or, "and": set_and, "union": None, "intersection": None,
    "equal": equal, "neq": neq, "lt": lt, "lte": lte, "gt": gt, "gte": gte,
    "startswith": startswith, "endswith": endswith, "contains": contains, "replace": replace,
    "substring": substring, "split": split, "concat": concat, "trim": trim, "trim_prefix": trim_prefix,
    "trim_suffix": trim_suffix, "lower": lower, "upper": upper, "indexof": indexof, "sprintf": sprintf,
    "re_match": re_match, "regex.match": re_match, "to_number": to_number,
    "is_number": is_number, "is_string": is_string, "is_boolean": is_boolean, "is_array": is_array,
    "is_set": is_set, "is_object": is_object, "is_null": is_null, "type_name": type_name, "sort": sort,
    "array.concat": array_concat,
}
BUILTINS = {k: v for k, v in BUILTINS.items() if v is not None}

ARITY = {
    "count": 1, "any": 1, "all": 1, "sum": 1, "max": 1, "min": 1, "plus": 2, "minus": 2, "mul": 2, "div": 2,
    "rem": 2, "abs": 1, "or": 2, "and": 2, "equal": 2, "neq": 2, "lt": 2, "lte": 2, "gt": 2, "gte": 2,
    "startswith": 2, "endswith": 2, "contains": 2, "replace": 3, "substring": 3, "split": 2, "concat": 2,
    "trim": 2, "trim_prefix": 2, "trim_suffix": 2, "lower": 1, "upper": 1, "indexof": 2, "sprintf": 2,
    "re_match": 2, "regex.match": 2, "to_number": 1, "is_number": 1, "is_string": 1, "is_boolean": 1,
    "is_array": 1, "is_set": 1, "is_object": 1, "is_null": 1, "type_name": 1, "sort": 1, "array.concat": 2,
}
