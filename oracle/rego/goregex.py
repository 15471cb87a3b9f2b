"""Go RE2 (regexp, Go 1.15) semantics on top of Python ``re`` — oracle only.

``re_match`` (``vendor/github.com/open-policy-agent/opa/topdown/regex.go:21-34``)
compiles with Go's ``regexp.Compile`` and runs an unanchored search.  Parity is
UNPINNED: the reference holds no regex test vectors.  The
translation below covers the syntax the workloads use and refuses the rest:

* ``$`` (no ``(?m)``) is end-of-text (Python ``\\Z``), ``\\z`` likewise;
* ``\\d \\w \\s \\b`` are ASCII (``re.ASCII``);
* ``.`` excludes ``\\n`` unless ``(?s)``;
* back-references and look-around are compile errors in Go -> RegoError;
* Unicode classes ``\\p{..}``, ``\\Q..\\E``, ``(?U)`` raise NotImplementedError.
"""
from __future__ import annotations

import re

from .values import RegoError

_CACHE = {}


def compile_go(pattern: str):
    got = _CACHE.get(pattern)
    if got is not None:
        return got
    py = _translate(pattern)
    try:
        rx = re.compile(py, re.ASCII)
    except re.error as e:  # pragma: no cover - translation guards most cases
        raise RegoError("error parsing regexp: %s" % e)
    _CACHE[pattern] = rx
    return rx


def _translate(p: str) -> str:
    out = []
    i = 0
    n = len(p)
    in_class = False
    multiline = False
    while i < n:
        c = p[i]
        if c == "\\":
            if i + 1 >= n:
                raise RegoError("error parsing regexp: trailing backslash at end of expression")
            d = p[i + 1]
            if d.isdigit() and d != "0" and not in_class:
                raise RegoError("error parsing regexp: invalid escape sequence: `\\%s`" % d)
            if d in "pPQE":
                raise NotImplementedError("unicode class / quoting in regex")
            if d == "z" and not in_class:
                out.append(r"\Z")
            elif d == "Z":
                raise RegoError("error parsing regexp: invalid escape sequence: `\\Z`")
            else:
                out.append(c + d)
            i += 2
            continue
        if in_class:
            if c == "[" and p.startswith("[:", i):
                raise NotImplementedError("POSIX class")
            if c == "]":
                in_class = False
            out.append(c)
            i += 1
            continue
        if c == "[":
            in_class = True
            out.append(c)
            i += 1
            # a leading ']' or '^]' is literal
            if i < n and p[i] == "^":
                out.append("^")
                i += 1
            if i < n and p[i] == "]":
                out.append(r"\]")
                i += 1
            continue
        if c == "(" and p.startswith("(?", i):
            if p.startswith("(?=", i) or p.startswith("(?!", i) or p.startswith("(?<=", i) or p.startswith("(?<!", i):
                raise RegoError("error parsing regexp: invalid or unsupported Perl syntax")
            if p.startswith("(?P<", i):
                out.append("(?P<")
                i += 4
                continue
            m = re.match(r"\(\?([imsU-]*)(\)|:)", p[i:])
            if not m:
                raise RegoError("error parsing regexp: invalid or unsupported Perl syntax")
            flags = m.group(1)
            if "U" in flags:
                raise NotImplementedError("(?U)")
            if "m" in flags.split("-")[0]:
                multiline = True
            out.append(m.group(0))
            i += len(m.group(0))
            continue
        if c == "$":
            out.append("$" if multiline else r"\Z")
            i += 1
            continue
        if c == "{":
            m = re.match(r"\{(\d+)(,(\d*))?\}", p[i:])
            if m:
                lo = int(m.group(1))
                hi = m.group(3)
                if lo > 1000 or (hi not in (None, "") and int(hi) > 1000):
                    raise RegoError("error parsing regexp: invalid repeat count")
        out.append(c)
        i += 1
    if in_class:
        raise RegoError("error parsing regexp: missing closing ]")
    return "".join(out)


def re_match(pattern: str, value: str) -> bool:
    return compile_go(pattern).search(value) is not None
