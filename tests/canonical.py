"""Canonical comparison of violation messages that print Rego objects or sets.

OPA v0.21 prints an object in its insertion order, and objects converted from
Go maps (the review, constraint parameters) are filled in Go map iteration
order, which is random per run (vendor/.../opa/ast/term.go:79-92, SURVEY.md
8(c)).  So a message that %v-prints an object -- the PSP templates print
`input.parameters`, a container's `securityContext`, a `volume` -- has no
single reference byte string.  The engine prints members in document (JSON
source) order; that is a deterministic choice among the reference's possible
outputs.  For those messages parity is checked after canonicalising every
printed object / set term: members sorted by their canonical text.  Messages
without such terms compare byte for byte (canonicalisation is the identity on
them).
"""
from __future__ import annotations

import json


class _P:
    def __init__(self, s, i):
        self.s, self.i = s, i

    def ws(self):
        while self.i < len(self.s) and self.s[self.i] == " ":
            self.i += 1

    def peek(self):
        return self.s[self.i] if self.i < len(self.s) else ""


def _string(p):
    """a Go strconv.Quote'd string; its canonical text is the quoted text"""
    j = p.i + 1
    while j < len(p.s):
        if p.s[j] == "\\":
            j += 2
            continue
        if p.s[j] == '"':
            break
        j += 1
    if j >= len(p.s):
        raise ValueError("unterminated string")
    lit = p.s[p.i:j + 1]
    p.i = j + 1
    return lit


def _term(p, depth=0):
    """parse one printed Rego term at p.i; returns its canonical text"""
    if depth > 64:
        raise ValueError("too deep")
    p.ws()
    c = p.peek()
    if c == '"':
        return _string(p)
    if p.s.startswith("set()", p.i):
        p.i += 5
        return "set()"
    if c == "[":
        p.i += 1
        items = []
        p.ws()
        if p.peek() == "]":
            p.i += 1
            return "[]"
        while True:
            items.append(_term(p, depth + 1))
            p.ws()
            if p.peek() == ",":
                p.i += 1
                continue
            if p.peek() == "]":
                p.i += 1
                return "[" + ", ".join(items) + "]"
            raise ValueError("bad array")
    if c == "{":
        p.i += 1
        p.ws()
        if p.peek() == "}":
            p.i += 1
            return "{}"
        members, is_obj = [], None
        while True:
            k = _term(p, depth + 1)
            p.ws()
            if p.peek() == ":":
                if is_obj is False:
                    raise ValueError("mixed set/object")
                is_obj = True
                p.i += 1
                v = _term(p, depth + 1)
                members.append(k + ": " + v)
            else:
                if is_obj is True:
                    raise ValueError("mixed set/object")
                is_obj = False
                members.append(k)
            p.ws()
            if p.peek() == ",":
                p.i += 1
                continue
            if p.peek() == "}":
                p.i += 1
                return "{" + ", ".join(sorted(members)) + "}"
            raise ValueError("bad object/set")
    # scalars: numbers, true / false / null
    j = p.i
    while j < len(p.s) and (p.s[j].isalnum() or p.s[j] in "+-.eE_"):
        j += 1
    if j == p.i:
        raise ValueError("no term")
    tok = p.s[p.i:j]
    if tok not in ("true", "false", "null"):
        json.loads(tok)  # a number, or not a term
    p.i = j
    return tok


def canonical_message(msg: str) -> str:
    """msg with every printed object / set term's members sorted"""
    out, i = [], 0
    while i < len(msg):
        c = msg[i]
        if c == "{" or (c == "s" and msg.startswith("set()", i)):
            p = _P(msg, i)
            try:
                t = _term(p)
                out.append(t)
                i = p.i
                continue
            except (ValueError, json.JSONDecodeError):
                pass
        out.append(c)
        i += 1
    return "".join(out)


def canonical_row(row):
    """(kind, name, msg, details, EA) with the message canonicalised"""
    if isinstance(row, tuple) and len(row) >= 3:
        return row[:2] + (canonical_message(row[2]),) + row[3:]
    return row
