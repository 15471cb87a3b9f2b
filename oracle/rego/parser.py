"""Rego (OPA v0.21 subset) lexer + parser for the oracle — test infrastructure only.

Covers the language used by the Gatekeeper target library
(``pkg/target/regolib/src.rego``), its ``*_test.rego`` KATs, the frameworks
hooks (``vendor/.../frameworks/constraint/pkg/client/regolib/src.go``) and the
ConstraintTemplates of the BASELINE workloads: packages, imports, complete /
partial-set / partial-object / function rules, ``default``, bodies with
``not``, ``some``, ``with``, ``:=`` / ``=`` / comparison / arithmetic / set
infix operators, refs, calls, array/object/set literals and comprehensions.
Precedence follows OPA's grammar (relation < ``|`` < ``&`` < ``+ -`` < ``* / %``).
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from typing import List, Optional

from .values import Num, NULL

# --------------------------------------------------------------------------
# AST
# --------------------------------------------------------------------------


@dataclass(eq=False)
class Scalar:
    value: object


@dataclass(eq=False)
class Var:
    name: str


@dataclass(eq=False)
class Ref:
    head: object  # Var or Call
    path: list  # list of terms (string Scalars for .field)


@dataclass(eq=False)
class ArrayT:
    items: list


@dataclass(eq=False)
class ObjectT:
    pairs: list  # list of (key term, value term)


@dataclass(eq=False)
class SetT:
    items: list


@dataclass(eq=False)
class ArrayCompr:
    term: object
    body: list


@dataclass(eq=False)
class SetCompr:
    term: object
    body: list


@dataclass(eq=False)
class ObjectCompr:
    key: object
    value: object
    body: list


@dataclass(eq=False)
class Call:
    op: list  # name path, e.g. ["count"] or ["data","lib","f"] or ["plus"]
    args: list


@dataclass(eq=False)
class With:
    target: object  # Ref/Var term
    value: object


@dataclass(eq=False)
class Expr:
    kind: str  # 'term' | 'assign' | 'unify' | 'some'
    terms: list
    negated: bool = False
    withs: list = field(default_factory=list)
    loc: int = 0


@dataclass(eq=False)
class Rule:
    name: str
    kind: str  # 'complete' | 'partial_set' | 'partial_obj' | 'func'
    key: object = None
    value: object = None
    args: list = None
    body: list = None
    default: bool = False
    package: tuple = ()
    module: object = None
    is_else: bool = False


@dataclass(eq=False)
class Module:
    package: tuple
    imports: list
    rules: list


# --------------------------------------------------------------------------
# lexer
# --------------------------------------------------------------------------

_TOKEN_RE = re.compile(
    r"""
    (?P<ws>[ \t\r]+)
  | (?P<comment>\#[^\n]*)
  | (?P<nl>\n)
  | (?P<rawstr>`[^`]*`)
  | (?P<str>"(?:[^"\\\n]|\\.)*")
  | (?P<num>(?:0|[1-9][0-9]*)(?:\.[0-9]+)?(?:[eE][+-]?[0-9]+)?)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
  | (?P<op>:=|==|!=|<=|>=|[{}\[\]().,;:=<>+\-*/%|&])
    """,
    re.VERBOSE,
)


@dataclass
class Tok:
    kind: str
    text: str
    pos: int


def lex(src: str) -> List[Tok]:
    toks = []
    i = 0
    n = len(src)
    while i < n:
        m = _TOKEN_RE.match(src, i)
        if not m:
            raise SyntaxError("rego lex error at %d: %r" % (i, src[i:i + 20]))
        kind = m.lastgroup
        text = m.group(kind)
        if kind not in ("ws", "comment"):
            toks.append(Tok(kind, text, i))
        i = m.end()
    toks.append(Tok("eof", "", n))
    return toks


def _unquote(s: str) -> str:
    if s.startswith("`"):
        return s[1:-1]
    # Go string literal escapes == JSON escapes for the subset used
    return json.loads(s)


# --------------------------------------------------------------------------
# parser
# --------------------------------------------------------------------------

KEYWORDS = {"package", "import", "not", "with", "as", "default", "some", "else", "true", "false", "null"}

INFIX = {
    "==": "equal", "!=": "neq", "<": "lt", "<=": "lte", ">": "gt", ">=": "gte",
    "|": "or", "&": "and", "+": "plus", "-": "minus", "*": "mul", "/": "div", "%": "rem",
}
LEVELS = [("==", "!=", "<", "<=", ">", ">="), ("|",), ("&",), ("+", "-"), ("*", "/", "%")]


class Parser:
    def __init__(self, src: str):
        self.toks = lex(src)
        self.i = 0
        self.wild = 0
        self.nl_sensitive = [False]

    # -- token helpers --------------------------------------------------
    def peek(self, k=0) -> Tok:
        j = self.i
        cnt = 0
        while True:
            t = self.toks[j]
            if t.kind == "nl" and not self.nl_sensitive[-1]:
                j += 1
                continue
            if cnt == k:
                return t
            cnt += 1
            j += 1

    def next(self) -> Tok:
        while self.toks[self.i].kind == "nl" and not self.nl_sensitive[-1]:
            self.i += 1
        t = self.toks[self.i]
        self.i += 1
        return t

    def skip_nl(self):
        while self.toks[self.i].kind == "nl":
            self.i += 1

    def at(self, text) -> bool:
        t = self.peek()
        return t.kind in ("op", "ident") and t.text == text

    def expect(self, text) -> Tok:
        t = self.next()
        if t.text != text:
            raise SyntaxError("expected %r got %r at %d" % (text, t.text, t.pos))
        return t

    def fresh_wild(self) -> Var:
        self.wild += 1
        return Var("$_%d" % self.wild)

    # -- module -----------------------------------------------------------
    def parse_module(self) -> Module:
        self.nl_sensitive = [False]
        self.expect("package")
        pkg = self.parse_ref_path()
        imports = []
        rules = []
        while self.peek().kind != "eof":
            if self.at("import"):
                self.next()
                path = self.parse_ref_path()
                alias = None
                if self.at("as"):
                    self.next()
                    alias = self.next().text
                imports.append((path, alias or path[-1]))
                continue
            rules.extend(self.parse_rule(tuple(pkg)))
        mod = Module(tuple(pkg), imports, rules)
        for r in rules:
            r.module = mod
        return mod

    def parse_ref_path(self) -> list:
        t = self.next()
        if t.kind != "ident":
            raise SyntaxError("expected identifier at %d" % t.pos)
        path = [t.text]
        while True:
            nt = self.toks[self.i]
            if nt.kind == "op" and nt.text == ".":
                self.i += 1
                path.append(self.next().text)
            elif nt.kind == "op" and nt.text == "[":
                self.i += 1
                s = self.next()
                path.append(_unquote(s.text))
                self.expect("]")
            else:
                break
        return path

    def parse_rule(self, pkg) -> List[Rule]:
        default = False
        if self.at("default"):
            self.next()
            default = True
        name = self.next()
        if name.kind != "ident":
            raise SyntaxError("expected rule name at %d got %r" % (name.pos, name.text))
        r = Rule(name=name.text, kind="complete", package=pkg, default=default)
        if self.at("("):
            self.next()
            args = []
            while not self.at(")"):
                args.append(self.parse_term())
                if self.at(","):
                    self.next()
            self.expect(")")
            r.kind = "func"
            r.args = args
        elif self.at("["):
            self.next()
            r.key = self.parse_term()
            self.expect("]")
            r.kind = "partial_set"
        if self.at("=") or self.at(":="):
            self.next()
            r.value = self.parse_term()
            if r.kind == "partial_set":
                r.kind = "partial_obj"
        if default:
            r.body = []
            return [r]
        rules = []
        if self.at("{"):
            r.body = self.parse_body_braced()
        else:
            r.body = []  # constant rule `x = 1` or `p[x]`-less
        rules.append(r)
        # else chains: `else = v { body }`
        while self.at("else"):
            self.next()
            er = Rule(name=r.name, kind=r.kind, key=r.key, args=r.args, package=pkg, is_else=True)
            if self.at("=") or self.at(":="):
                self.next()
                er.value = self.parse_term()
            else:
                er.value = Scalar(True)
            er.body = self.parse_body_braced() if self.at("{") else []
            rules.append(er)
        if r.kind == "complete" and r.value is None:
            r.value = Scalar(True)
        if r.kind == "func" and r.value is None:
            r.value = Scalar(True)
        return rules

    # -- bodies -------------------------------------------------------------
    def parse_body_braced(self) -> list:
        self.expect("{")
        self.nl_sensitive.append(True)
        body = self.parse_body_until("}")
        self.expect("}")
        self.nl_sensitive.pop()
        return body

    def parse_body_until(self, closer) -> list:
        body = []
        while True:
            self.skip_nl()
            t = self.toks[self.i]
            if t.kind == "op" and t.text == closer:
                break
            if t.kind == "op" and t.text == ";":
                self.i += 1
                continue
            body.append(self.parse_expr())
            # expression terminator: newline, ';' or closer
            t = self.toks[self.i]
            if t.kind == "nl" or (t.kind == "op" and t.text in (";", closer)):
                continue
            raise SyntaxError("unexpected %r at %d" % (t.text, t.pos))
        return body

    def parse_expr(self) -> Expr:
        pos = self.peek().pos
        if self.at("some"):
            self.next()
            names = [self.parse_term()]
            while self.at(","):
                self.next()
                names.append(self.parse_term())
            return Expr("some", names, loc=pos)
        negated = False
        if self.at("not"):
            self.next()
            negated = True
        lhs = self.parse_term()
        if self.at(":="):
            self.next()
            rhs = self.parse_term()
            e = Expr("assign", [lhs, rhs], negated=negated, loc=pos)
        elif self.at("="):
            self.next()
            rhs = self.parse_term()
            e = Expr("unify", [lhs, rhs], negated=negated, loc=pos)
        else:
            e = Expr("term", [lhs], negated=negated, loc=pos)
        while self._with_follows():
            self.skip_nl()
            self.next()
            target = self.parse_term()
            self.expect("as")
            value = self.parse_term()
            e.withs.append(With(target, value))
        return e

    def _with_follows(self):
        j = self.i
        while self.toks[j].kind == "nl":
            j += 1
        t = self.toks[j]
        return t.kind == "ident" and t.text == "with"

    # -- terms ---------------------------------------------------------------
    def parse_term(self, level=0):
        if level == len(LEVELS):
            return self.parse_unary()
        lhs = self.parse_term(level + 1)
        while True:
            t = self.peek()
            # infix operators never span a newline inside a braced body
            if t.kind == "op" and t.text in LEVELS[level]:
                self.next()
                self.skip_nl_if_insensitive()
                rhs = self.parse_term(level + 1)
                lhs = Call([INFIX[t.text]], [lhs, rhs])
            else:
                break
        return lhs

    def skip_nl_if_insensitive(self):
        while self.toks[self.i].kind == "nl":
            self.i += 1

    def parse_unary(self):
        t = self.peek()
        if t.kind == "op" and t.text == "-":
            nt = self.peek(1)
            if nt.kind == "num":
                self.next()
                self.next()
                return Scalar(Num("-" + nt.text))
            self.next()
            operand = self.parse_unary()
            return Call(["minus"], [Scalar(Num("0")), operand])
        return self.parse_postfix()

    def parse_postfix(self):
        prim = self.parse_primary()
        path = []
        head = prim
        while True:
            t = self.peek()
            if t.kind == "op" and t.text == "." :
                self.next()
                f = self.next()
                path.append(Scalar(f.text))
            elif t.kind == "op" and t.text == "[":
                self.next()
                self.nl_sensitive.append(False)
                sel = self.parse_term()
                self.expect("]")
                self.nl_sensitive.pop()
                path.append(sel)
            elif t.kind == "op" and t.text == "(" and isinstance(head, (Var,)) :
                # call: op path is head + dotted path so far
                names = [head.name] + [p.value for p in path]
                if any(not isinstance(p, Scalar) for p in path):
                    raise SyntaxError("dynamic call target")
                self.next()
                self.nl_sensitive.append(False)
                args = []
                while not self.at(")"):
                    args.append(self.parse_term())
                    if self.at(","):
                        self.next()
                self.expect(")")
                self.nl_sensitive.pop()
                head = Call(names, args)
                path = []
            else:
                break
        if not path:
            return head
        return Ref(head, path)

    def parse_primary(self):
        t = self.next()
        if t.kind == "num":
            return Scalar(Num(t.text))
        if t.kind in ("str", "rawstr"):
            return Scalar(_unquote(t.text))
        if t.kind == "ident":
            if t.text == "true":
                return Scalar(True)
            if t.text == "false":
                return Scalar(False)
            if t.text == "null":
                return Scalar(NULL)
            if t.text == "_":
                return self.fresh_wild()
            return Var(t.text)
        if t.kind == "op" and t.text == "(":
            self.nl_sensitive.append(False)
            inner = self.parse_term()
            self.expect(")")
            self.nl_sensitive.pop()
            return inner
        if t.kind == "op" and t.text == "[":
            return self.parse_array_or_compr()
        if t.kind == "op" and t.text == "{":
            return self.parse_brace()
        raise SyntaxError("unexpected token %r at %d" % (t.text, t.pos))

    def parse_array_or_compr(self):
        self.nl_sensitive.append(False)
        if self.at("]"):
            self.next()
            self.nl_sensitive.pop()
            return ArrayT([])
        first = self._parse_compr_head()
        if self._at_compr_bar():
            self.next()
            self.nl_sensitive.pop()
            self.nl_sensitive.append(True)
            body = self.parse_body_until("]")
            self.expect("]")
            self.nl_sensitive.pop()
            return ArrayCompr(first, body)
        items = [first]
        while self.at(","):
            self.next()
            if self.at("]"):
                break
            items.append(self.parse_term())
        self.expect("]")
        self.nl_sensitive.pop()
        return ArrayT(items)

    def _at_compr_bar(self):
        return self.at("|")

    def parse_brace(self):
        self.nl_sensitive.append(False)
        if self.at("}"):
            self.next()
            self.nl_sensitive.pop()
            return ObjectT([])
        first = self._parse_compr_head()
        if self.at(":"):
            self.next()
            val = self._parse_compr_head()
            if self.at("|"):
                self.next()
                self.nl_sensitive.pop()
                self.nl_sensitive.append(True)
                body = self.parse_body_until("}")
                self.expect("}")
                self.nl_sensitive.pop()
                return ObjectCompr(first, val, body)
            pairs = [(first, val)]
            while self.at(","):
                self.next()
                if self.at("}"):
                    break
                k = self.parse_term()
                self.expect(":")
                v = self.parse_term()
                pairs.append((k, v))
            self.expect("}")
            self.nl_sensitive.pop()
            return ObjectT(pairs)
        if self.at("|"):
            self.next()
            self.nl_sensitive.pop()
            self.nl_sensitive.append(True)
            body = self.parse_body_until("}")
            self.expect("}")
            self.nl_sensitive.pop()
            return SetCompr(first, body)
        items = [first]
        while self.at(","):
            self.next()
            if self.at("}"):
                break
            items.append(self.parse_term())
        self.expect("}")
        self.nl_sensitive.pop()
        return SetT(items)

    def _parse_compr_head(self):
        # A comprehension head is a term that may not use the top-level `|`
        # operator (OPA disambiguates the same way).
        return self._parse_no_bar(0)

    def _parse_no_bar(self, level):
        if level == len(LEVELS):
            return self.parse_unary()
        if LEVELS[level] == ("|",):
            return self._parse_no_bar(level + 1)
        lhs = self._parse_no_bar(level + 1)
        while True:
            t = self.peek()
            if t.kind == "op" and t.text in LEVELS[level]:
                self.next()
                rhs = self._parse_no_bar(level + 1)
                lhs = Call([INFIX[t.text]], [lhs, rhs])
            else:
                break
        return lhs


def parse_module(src: str) -> Module:
    p = Parser(src)
    return p.parse_module()

