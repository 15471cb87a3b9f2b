"""Go RE2 (regexp, Go 1.15) semantics on top of Python ``re`` — oracle only.

``re_match`` (``vendor/github.com/open-policy-agent/opa/topdown/regex.go:21-34``)
compiles with Go's ``regexp.Compile`` and runs an unanchored search.  Parity is
UNPINNED: the reference holds no regex test vectors; the rules
below restate Go's documented syntax (regexp/syntax) and are checked by the
known answers in ``tests/test_go_regex.py``.  The translation covers the
syntax the workloads use and refuses the rest:

* ``$`` (no ``(?m)``) is end-of-text (Python ``\\Z``), ``\\z`` likewise;
* ``\\d \\w \\b`` are ASCII (``re.ASCII``); ``\\s`` is Go's ``[\\t\\n\\f\\r ]``
  (Python's ASCII ``\\s`` also holds ``\\v``), ``\\S`` its complement;
* ``(?i)`` is Go's simple case folding: ASCII letters pair up, and k/K also
  fold with U+212A (KELVIN SIGN), s/S with U+017F (LATIN SMALL LETTER LONG S)
  -- Python's ASCII folding has neither, its Unicode folding also pairs i
  with U+0130/U+0131, which Go does not.  Letters, ``\\w`` / ``\\W`` and
  classes under ``(?i)`` are written out with those two code points;
* flags set mid-group (``a(?i)b``) apply to the rest of the group, as in Go
  (Python 3.10 would apply them to the whole pattern): they become a scoped
  group ``(?i:...)`` closed with the enclosing group;
* ``.`` excludes ``\\n`` unless ``(?s)``;
* back-references and look-around are compile errors in Go -> RegoError;
* Unicode classes ``\\p{..}``, ``\\Q..\\E``, ``(?U)``, hex escapes under
  ``(?i)`` and ``\\S`` inside a class raise NotImplementedError.
"""
from __future__ import annotations

import re

from .values import RegoError

_CACHE = {}

_KELVIN, _LONG_S = "\u212a", "\u017f"
_SPACE = r"\t\n\x0c\r "  # Go's \s (regexp/syntax perl_groups.go)


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


def _fold_extra(body: str) -> str:
    """the non-ASCII fold partners Go adds to a class `[body]` under (?i)"""
    rx = re.compile("[" + body + "]", re.ASCII | re.IGNORECASE)
    return (_KELVIN if rx.match("k") else "") + (_LONG_S if rx.match("s") else "")


def _flags(spec: str, icase: bool) -> bool:
    """(?spec...): the case-folding state after it"""
    on, _, off = spec.partition("-")
    if "i" in on:
        icase = True
    if "i" in off:
        icase = False
    return icase


def _translate(p: str) -> str:
    out = []
    i = 0
    n = len(p)
    multiline = False
    icase = False
    # open groups: [case-folding state to restore, the flag specs of
    # mid-group changes whose scoped groups it owes a ')'] -- the bottom entry
    # is the pattern itself; an alternation closes and reopens them, since a
    # change holds in the group's later branches too
    groups = [[False, []]]
    while i < n:
        c = p[i]
        if c == "\\":
            if i + 1 >= n:
                raise RegoError("error parsing regexp: trailing backslash at end of expression")
            d = p[i + 1]
            if d.isdigit() and d != "0":
                raise RegoError("error parsing regexp: invalid escape sequence: `\\%s`" % d)
            if d in "pPQE":
                raise NotImplementedError("unicode class / quoting in regex")
            if d == "x" and icase:
                raise NotImplementedError("hex escape under (?i)")
            if d == "z":
                out.append(r"\Z")
            elif d == "Z":
                raise RegoError("error parsing regexp: invalid escape sequence: `\\Z`")
            elif d == "s":
                out.append("[" + _SPACE + "]")
            elif d == "S":
                out.append("[^" + _SPACE + "]")
            elif d == "w" and icase:
                out.append(r"[\w" + _KELVIN + _LONG_S + "]")
            elif d == "W" and icase:
                out.append(r"[^\w" + _KELVIN + _LONG_S + "]")
            else:
                out.append(c + d)
            i += 2
            continue
        if c == "[":
            i += 1
            neg = False
            if i < n and p[i] == "^":
                neg = True
                i += 1
            body = []
            first = True
            while True:
                if i >= n:
                    raise RegoError("error parsing regexp: missing closing ]")
                ch = p[i]
                if ch == "]" and not first:
                    i += 1
                    break
                first = False
                if ch == "[" and p.startswith("[:", i):
                    raise NotImplementedError("POSIX class")
                if ch == "\\":
                    if i + 1 >= n:
                        raise RegoError("error parsing regexp: missing closing ]")
                    d = p[i + 1]
                    if d in "pPQE":
                        raise NotImplementedError("unicode class / quoting in regex")
                    if d == "S":
                        raise NotImplementedError(r"\S inside a class")
                    if d == "x" and icase:
                        raise NotImplementedError("hex escape under (?i)")
                    body.append(_SPACE if d == "s" else ch + d)
                    i += 2
                    continue
                body.append(r"\]" if ch == "]" else r"\[" if ch == "[" else ch)
                i += 1
            text = "".join(body)
            if icase:
                text += _fold_extra(text)
            out.append("[" + ("^" if neg else "") + text + "]")
            continue
        if c == "(":
            if p.startswith("(?=", i) or p.startswith("(?!", i) or p.startswith("(?<=", i) or p.startswith("(?<!", i):
                raise RegoError("error parsing regexp: invalid or unsupported Perl syntax")
            if p.startswith("(?P<", i):
                e = p.find(">", i)
                if e < 0:
                    raise RegoError("error parsing regexp: invalid named capture")
                groups.append([icase, []])
                out.append(p[i:e + 1])  # the name verbatim
                i = e + 1
                continue
            if p.startswith("(?", i):
                m = re.match(r"\(\?([imsU-]*)(\)|:)", p[i:])
                if not m or (m.group(1) == "" and m.group(2) == ")"):
                    raise RegoError("error parsing regexp: invalid or unsupported Perl syntax")
                spec = m.group(1)
                if "U" in spec:
                    raise NotImplementedError("(?U)")
                if "m" in spec.split("-")[0]:
                    multiline = True
                i += len(m.group(0))
                if m.group(2) == ")":
                    # a flag change for the rest of the enclosing group
                    out.append("(?" + spec + ":")
                    groups[-1][1].append(spec)
                    icase = _flags(spec, icase)
                else:
                    groups.append([icase, []])
                    out.append("(?" + spec + ":")
                    icase = _flags(spec, icase)
                continue
            groups.append([icase, []])
            out.append("(")
            i += 1
            continue
        if c == ")":
            if len(groups) == 1:
                raise RegoError("error parsing regexp: unexpected )")
            saved, owed = groups.pop()
            out.append(")" * len(owed) + ")")
            icase = saved
            i += 1
            continue
        if c == "|" and groups[-1][1]:
            specs = groups[-1][1]
            out.append(")" * len(specs) + "|" + "".join("(?" + f + ":" for f in specs))
            i += 1
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
        if icase and c in "kKsS":
            out.append("[" + c.lower() + c.upper() + (_KELVIN if c in "kK" else _LONG_S) + "]")
            i += 1
            continue
        out.append(c)
        i += 1
    if len(groups) > 1:
        raise RegoError("error parsing regexp: missing closing )")
    out.append(")" * len(groups[0][1]))
    return "".join(out)


def re_match(pattern: str, value: str) -> bool:
    return compile_go(pattern).search(value) is not None
