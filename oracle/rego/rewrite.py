"""Body rewrites OPA's compiler applies before evaluation — oracle restatement.

Two stages of ``vendor/github.com/open-policy-agent/opa/ast/compile.go`` change
observable semantics inside negated expressions, so the oracle reproduces them:

* ``RewriteExprTerms`` (expandExpr / expandExprTerm): calls nested inside other
  terms are hoisted into their own (non-negated) expressions with an output
  variable, e.g. ``not f(g(x))`` -> ``g(x, $l0); not f($l0)``;
* ``RewriteDynamicTerms`` (``compile.go:2828-2960``, after safety reordering):
  ref arguments of call expressions and ref-valued ref selectors are hoisted
  into ``$lN = ref`` expressions placed before the original, e.g.
  ``not re_match(e.allowedRegex, v)`` -> ``$l1 = e.allowedRegex; not re_match($l1, v)``
  and ``not data.x[input.ns]`` -> ``$l2 = input.ns; not data.x[$l2]``.
"""
from __future__ import annotations

import itertools

from .parser import ArrayCompr, ArrayT, Call, Expr, ObjectCompr, ObjectT, Ref, Scalar, SetCompr, SetT, Var

_gen = itertools.count()


def _fresh():
    return Var("$l%d" % next(_gen))


# ---------------------------------------------------------------------------
# RewriteExprTerms
# ---------------------------------------------------------------------------


def expand_body(body):
    out = []
    for e in body:
        out.extend(expand_expr(e))
    return out


def expand_expr(e: Expr):
    if e.kind == "some":
        return [e]
    support = []
    if e.kind == "term":
        t = e.terms[0]
        if isinstance(t, Call):
            args = []
            for a in t.args:
                s, a2 = _expand_term(a)
                support += s
                args.append(a2)
            new = Expr("term", [Call(t.op, args)], negated=e.negated, withs=e.withs, loc=e.loc)
        else:
            s, t2 = _expand_top(t)
            support += s
            new = Expr("term", [t2], negated=e.negated, withs=e.withs, loc=e.loc)
    else:
        terms = []
        for t in e.terms:
            s, t2 = _expand_term(t)
            support += s
            terms.append(t2)
        new = Expr(e.kind, terms, negated=e.negated, withs=e.withs, loc=e.loc)
    for s in support:
        s.withs = e.withs
    return support + [new]


def _expand_top(t):
    if isinstance(t, Ref):
        return _expand_ref(t)
    return _expand_term(t)


def _expand_term(t):
    if isinstance(t, Call):
        support = []
        args = []
        for a in t.args:
            s, a2 = _expand_term(a)
            support += s
            args.append(a2)
        v = _fresh()
        support.append(Expr("term", [Call(t.op, args + [v])]))
        return support, v
    if isinstance(t, Ref):
        return _expand_ref(t)
    if isinstance(t, ArrayT):
        support, items = [], []
        for x in t.items:
            s, x2 = _expand_term(x)
            support += s
            items.append(x2)
        return support, ArrayT(items)
    if isinstance(t, SetT):
        support, items = [], []
        for x in t.items:
            s, x2 = _expand_term(x)
            support += s
            items.append(x2)
        return support, SetT(items)
    if isinstance(t, ObjectT):
        support, pairs = [], []
        for k, v in t.pairs:
            s1, k2 = _expand_term(k)
            s2, v2 = _expand_term(v)
            support += s1 + s2
            pairs.append((k2, v2))
        return support, ObjectT(pairs)
    if isinstance(t, ArrayCompr):
        s, term = _expand_term(t.term)
        return [], ArrayCompr(term, expand_body(list(t.body) + s))
    if isinstance(t, SetCompr):
        s, term = _expand_term(t.term)
        return [], SetCompr(term, expand_body(list(t.body) + s))
    if isinstance(t, ObjectCompr):
        s1, k = _expand_term(t.key)
        s2, v = _expand_term(t.value)
        return [], ObjectCompr(k, v, expand_body(list(t.body) + s1 + s2))
    return [], t


def _expand_ref(r: Ref):
    support = []
    path = []
    for p in r.path:
        s, p2 = _expand_term(p)
        support += s
        path.append(p2)
    head = r.head
    if isinstance(head, Call):
        s, hv = _expand_term(head)
        support += s
        head = hv
    return support, Ref(head, path)


# ---------------------------------------------------------------------------
# RewriteDynamicTerms
# ---------------------------------------------------------------------------


def rewrite_dynamics(body, is_global):
    out = []
    for e in body:
        if e.kind == "some":
            out.append(e)
            continue
        res = []
        if e.kind in ("assign", "unify"):
            l2 = _dyn_in_term(e, e.terms[0], res, is_global)
            r2 = _dyn_in_term(e, e.terms[1], res, is_global)
            new = Expr(e.kind, [l2, r2], negated=e.negated, withs=e.withs, loc=e.loc)
        elif isinstance(e.terms[0], Call):
            c = e.terms[0]
            args = [_dyn_one(e, a, res, is_global) for a in c.args]
            new = Expr("term", [Call(c.op, args)], negated=e.negated, withs=e.withs, loc=e.loc)
        else:
            t2 = _dyn_in_term(e, e.terms[0], res, is_global)
            new = Expr("term", [t2], negated=e.negated, withs=e.withs, loc=e.loc)
        out.extend(res)
        out.append(new)
    return out


def _is_ref(t, is_global):
    if isinstance(t, Var):
        return is_global(t.name)
    if isinstance(t, Ref):
        return HOIST_LOCAL or (isinstance(t.head, Var) and is_global(t.head.name))
    return False


HOIST_LOCAL = False


def _dyn_in_term(orig, t, res, is_global):
    if isinstance(t, Ref):
        return Ref(t.head, [_dyn_one(orig, p, res, is_global) for p in t.path])
    if isinstance(t, ArrayCompr):
        return ArrayCompr(t.term, rewrite_dynamics(t.body, is_global))
    if isinstance(t, SetCompr):
        return SetCompr(t.term, rewrite_dynamics(t.body, is_global))
    if isinstance(t, ObjectCompr):
        return ObjectCompr(t.key, t.value, rewrite_dynamics(t.body, is_global))
    if isinstance(t, Var) and is_global(t.name):
        return t
    return _dyn_one(orig, t, res, is_global)


def _dyn_one(orig, t, res, is_global):
    if _is_ref(t, is_global):
        if isinstance(t, Ref):
            t = Ref(t.head, [_dyn_one(orig, p, res, is_global) for p in t.path])
        v = _fresh()
        res.append(Expr("unify", [v, t], withs=orig.withs))
        return v
    if isinstance(t, ArrayT):
        return ArrayT([_dyn_one(orig, x, res, is_global) for x in t.items])
    if isinstance(t, SetT):
        return SetT([_dyn_one(orig, x, res, is_global) for x in t.items])
    if isinstance(t, ObjectT):
        return ObjectT([(_dyn_one(orig, k, res, is_global), _dyn_one(orig, v, res, is_global)) for k, v in t.pairs])
    if isinstance(t, (ArrayCompr, SetCompr, ObjectCompr)):
        t2 = _dyn_in_term(orig, t, res, is_global)
        v = _fresh()
        res.append(Expr("unify", [v, t2], withs=orig.withs))
        return v
    return t
