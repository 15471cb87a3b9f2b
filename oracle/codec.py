"""Lossless JSON codec for oracle values in golden fixtures (test infrastructure).

Tags: {"#n": text} number, {"#o": [[k, v], ...]} object (insertion order, any
key type), {"#s": [...]} set, {"#u": 1} undefined; plain JSON for
null/bool/string/array.
"""
from __future__ import annotations

from .match import UNDEF
from .rego.values import NULL, Arr, Num, Obj, RSet


def enc(v):
    if v is UNDEF:
        return {"#u": 1}
    if v is NULL:
        return None
    if isinstance(v, bool) or isinstance(v, str):
        return v
    if isinstance(v, Num):
        return {"#n": v.text}
    if isinstance(v, Arr):
        return [enc(x) for x in v]
    if isinstance(v, RSet):
        return {"#s": [enc(x) for x in v]}
    if isinstance(v, Obj):
        return {"#o": [[enc(k), enc(x)] for k, x in v.items()]}
    raise TypeError(v)


def dec(x):
    if x is None:
        return NULL
    if isinstance(x, (bool, str)):
        return x
    if isinstance(x, list):
        return Arr(dec(e) for e in x)
    if isinstance(x, dict):
        if "#u" in x:
            return UNDEF
        if "#n" in x:
            return Num(x["#n"])
        if "#s" in x:
            return RSet(dec(e) for e in x["#s"])
        if "#o" in x:
            return Obj((dec(k), dec(v)) for k, v in x["#o"])
    raise TypeError(x)
