"""Top-down Rego evaluator for the oracle — test infrastructure only.

A restatement of OPA v0.21 ``topdown`` semantics for the subset the audit path
uses (``vendor/github.com/open-policy-agent/opa/topdown/eval.go``):

* bodies evaluate left to right after safety reordering
  (``ast/compiler.go`` reorderBodyForSafety);
* refs iterate unbound selector variables over object keys / array indices /
  set members;
* partial-set references with a key term are evaluated rule-by-rule and
  solution-by-solution without de-duplication (``evalVirtualPartial.evalOneRule``,
  eval.go:1867-1910); a full-extent reference builds the de-duplicated set
  (``evalAllRules``, eval.go:1839-1865);
* user functions yield at most once per call; a second solution with a
  different value is a conflict error; a ``false`` value of a function called
  as a statement is undefined (``evalFunc``, eval.go:1405-1497);
* complete rules with two different values are a conflict error;
* ``with`` replaces ``input`` / ``data`` subtrees for one expression;
* builtin failures raise :class:`RegoError` and abort the query
  (``topdown/builtins.go:145-164``).
"""
from __future__ import annotations

import itertools
from typing import Dict, List

from . import builtins as B
from .parser import (ArrayCompr, ArrayT, Call, Expr, Module, ObjectCompr, ObjectT, Ref, Rule, Scalar,
                     SetCompr, SetT, Var, parse_module)
from .rewrite import expand_body, rewrite_dynamics
from .values import NULL, Arr, ConflictError, Num, Obj, RegoError, RSet, rego_equal

_UNDEF = object()


class _PkgNode:
    __slots__ = ("children", "rules", "modules")

    def __init__(self):
        self.children: Dict[str, "_PkgNode"] = {}
        self.rules: Dict[str, List[Rule]] = {}
        self.modules: List[Module] = []


class Ctx:
    """Evaluation context: input + base data (+ caches), replaced by `with`."""

    __slots__ = ("input", "data", "cache")

    def __init__(self, input_val, data):
        self.input = input_val
        self.data = data
        self.cache = {}


class Env:
    __slots__ = ("ctx", "pkg", "module")

    def __init__(self, ctx, pkg, module):
        self.ctx = ctx
        self.pkg = pkg
        self.module = module


def _set_path(base, path, value):
    """Return a copy of `base` with `value` at `path` (creating objects)."""
    if not path:
        return value
    k = path[0]
    if not isinstance(base, Obj):
        base = Obj()
    child = base.get(k, _UNDEF)
    return base.with_item(k, _set_path(child if child is not _UNDEF else Obj(), path[1:], value))


class Interpreter:
    def __init__(self, modules=(), data=None, call_hook=None):
        self.root = _PkgNode()
        self.modules: List[Module] = []
        self.data = data if data is not None else Obj()
        self.call_hook = call_hook
        self._reorder_cache = {}
        for m in modules:
            self.add_module(m)

    # ------------------------------------------------------------------
    # module / data management
    # ------------------------------------------------------------------
    def add_module(self, m):
        if isinstance(m, str):
            m = parse_module(m)
        self.modules.append(m)
        node = self._pkg_node(m.package, create=True)
        node.modules.append(m)
        for r in m.rules:
            node.rules.setdefault(r.name, []).append(r)
        return m

    def remove_package(self, pkg):
        node = self._pkg_node(tuple(pkg), create=False)
        if node is None:
            return
        self.modules = [m for m in self.modules if m not in node.modules]
        node.modules = []
        node.rules = {}

    def _pkg_node(self, pkg, create=False):
        node = self.root
        for k in pkg:
            if k not in node.children:
                if not create:
                    return None
                node.children[k] = _PkgNode()
            node = node.children[k]
        return node

    # ------------------------------------------------------------------
    # public query API
    # ------------------------------------------------------------------
    def query_ref(self, path, input_val=_UNDEF):
        """All values of `data.<path>[x]` per solution (like `data.path[result]`)."""
        ctx = Ctx(input_val, self.data)
        env = Env(ctx, (), None)
        key = Var("$result")
        ref = Ref(Var("data"), [Scalar(p) for p in path] + [key])
        out = []
        for _, b in self.eval_term(ref, {}, env):
            out.append(b["$result"])
        return out

    def eval_rule_value(self, path, input_val=_UNDEF):
        ctx = Ctx(input_val, self.data)
        env = Env(ctx, (), None)
        ref = Ref(Var("data"), [Scalar(p) for p in path])
        return [v for v, _ in self.eval_term(ref, {}, env)]

    def run_test_rule(self, pkg, name):
        """Evaluate a `test_*` rule; returns True if defined and not false."""
        ctx = Ctx(_UNDEF, self.data)
        env = Env(ctx, tuple(pkg), None)
        vals = list(self.eval_term(Ref(Var("data"), [Scalar(p) for p in pkg] + [Scalar(name)]), {}, env))
        return bool(vals) and vals[0][0] is not False

    # ------------------------------------------------------------------
    # bodies and expressions
    # ------------------------------------------------------------------
    def eval_body(self, body, b, env, i=0):
        if i == len(body):
            yield b
            return
        for b2 in self.eval_expr(body[i], b, env):
            yield from self.eval_body(body, b2, env, i + 1)

    def _with_env(self, expr, b, env):
        inp = env.ctx.input
        data = env.ctx.data
        for w in expr.withs:
            vals = list(self.eval_term(w.value, b, env))
            if not vals:
                return None
            val = vals[0][0]
            path = self._with_path(w.target, b, env)
            if path[0] == "input":
                base = inp if inp is not _UNDEF else Obj()
                inp = _set_path(base, path[1:], val) if len(path) > 1 else val
            elif path[0] == "data":
                data = _set_path(data, path[1:], val)
            else:
                raise NotImplementedError("with target %r" % (path,))
        return Env(Ctx(inp, data), env.pkg, env.module)

    def _with_path(self, t, b, env):
        if isinstance(t, Var):
            return [t.name]
        if isinstance(t, Ref) and isinstance(t.head, Var):
            out = [t.head.name]
            for s in t.path:
                vs = list(self.eval_term(s, b, env))
                out.append(vs[0][0])
            return out
        raise NotImplementedError("with target")

    def eval_expr(self, e: Expr, b, env):
        if e.withs:
            env2 = self._with_env(e, b, env)
            if env2 is None:
                return
            env = env2
        if e.kind == "some":
            yield b
            return
        if e.negated:
            # OPA evaluates the whole negated body (evalNot), so errors anywhere
            # in it surface even after a first solution.
            found = False
            for _ in self._eval_expr_pos(e, b, env):
                found = True
            if not found:
                yield b
            return
        yield from self._eval_expr_pos(e, b, env)

    def _eval_expr_pos(self, e, b, env):
        if e.kind == "term":
            t = e.terms[0]
            if isinstance(t, Call):
                yield from self._eval_call_stmt(t, b, env)
                return
            for v, b2 in self.eval_term(t, b, env):
                if v is not False:
                    yield b2
            return
        if e.kind in ("assign", "unify"):
            yield from self.unify(e.terms[0], e.terms[1], b, env)
            return
        raise NotImplementedError(e.kind)

    def _eval_call_stmt(self, call: Call, b, env):
        for v, b2 in self.eval_call(call, b, env, statement=True):
            if v is not False:
                yield b2

    # ------------------------------------------------------------------
    # unification
    # ------------------------------------------------------------------
    def _is_unbound_var(self, t, b, env):
        return isinstance(t, Var) and t.name not in b and not self._is_global(t.name, env)

    def unify(self, a, c, b, env):
        if self._is_unbound_var(a, b, env):
            for v, b2 in self.eval_term(c, b, env):
                if a.name in b2:
                    if rego_equal(b2[a.name], v):
                        yield b2
                else:
                    b3 = dict(b2)
                    b3[a.name] = v
                    yield b3
            return
        if self._is_unbound_var(c, b, env):
            yield from self.unify(c, a, b, env)
            return
        if isinstance(a, ArrayT) and not self._ground(a, b, env):
            for v, b2 in self.eval_term(c, b, env):
                yield from self.unify_value(a, v, b2, env)
            return
        if isinstance(c, ArrayT) and not self._ground(c, b, env):
            for v, b2 in self.eval_term(a, b, env):
                yield from self.unify_value(c, v, b2, env)
            return
        if isinstance(a, ObjectT) and not self._ground(a, b, env):
            for v, b2 in self.eval_term(c, b, env):
                yield from self.unify_value(a, v, b2, env)
            return
        if isinstance(c, ObjectT) and not self._ground(c, b, env):
            for v, b2 in self.eval_term(a, b, env):
                yield from self.unify_value(c, v, b2, env)
            return
        for va, b2 in self.eval_term(a, b, env):
            for vc, b3 in self.eval_term(c, b2, env):
                if rego_equal(va, vc):
                    yield b3

    def unify_value(self, pat, v, b, env):
        """Unify a (possibly non-ground) pattern term with a value."""
        if self._is_unbound_var(pat, b, env):
            b2 = dict(b)
            b2[pat.name] = v
            yield b2
            return
        if isinstance(pat, Var) and pat.name in b:
            if rego_equal(b[pat.name], v):
                yield b
            return
        if isinstance(pat, ArrayT):
            if not isinstance(v, Arr) or len(v) != len(pat.items):
                return
            yield from self._unify_seq(list(zip(pat.items, v)), b, env)
            return
        if isinstance(pat, ObjectT):
            if not isinstance(v, Obj) or len(v) != len(pat.pairs):
                return
            pairs = []
            for kt, vt in pat.pairs:
                kvals = list(self.eval_term(kt, b, env))
                if len(kvals) != 1:
                    return
                k = kvals[0][0]
                if k not in v:
                    return
                pairs.append((vt, v.get(k)))
            yield from self._unify_seq(pairs, b, env)
            return
        for pv, b2 in self.eval_term(pat, b, env):
            if rego_equal(pv, v):
                yield b2

    def _unify_seq(self, pairs, b, env):
        if not pairs:
            yield b
            return
        (p, v), rest = pairs[0], pairs[1:]
        for b2 in self.unify_value(p, v, b, env):
            yield from self._unify_seq(rest, b2, env)

    def _ground(self, t, b, env):
        for name in _term_vars(t):
            if name not in b and not self._is_global(name, env):
                return False
        return True

    # ------------------------------------------------------------------
    # terms
    # ------------------------------------------------------------------
    def _is_global(self, name, env):
        if name in ("input", "data"):
            return True
        node = self._pkg_node(env.pkg)
        if node is not None and name in node.rules:
            return True
        if env.module is not None:
            for path, alias in env.module.imports:
                if alias == name:
                    return True
        return False

    def eval_term(self, t, b, env):
        """Yield (value, bindings) for every value of term t."""
        if isinstance(t, Scalar):
            yield t.value, b
            return
        if isinstance(t, Var):
            if t.name in b:
                yield b[t.name], b
                return
            yield from self._eval_ref_head(t.name, [], 0, b, env)
            return
        if isinstance(t, Ref):
            if isinstance(t.head, Var):
                if t.head.name in b:
                    yield from self.walk_value(b[t.head.name], t.path, 0, b, env)
                    return
                yield from self._eval_ref_head(t.head.name, t.path, 0, b, env)
                return
            for hv, b2 in self.eval_term(t.head, b, env):
                yield from self.walk_value(hv, t.path, 0, b2, env)
            return
        if isinstance(t, Call):
            yield from self.eval_call(t, b, env, statement=False)
            return
        if isinstance(t, ArrayT):
            yield from self._eval_seq(t.items, b, env, lambda vals: Arr(vals))
            return
        if isinstance(t, SetT):
            yield from self._eval_seq(t.items, b, env, lambda vals: RSet(vals))
            return
        if isinstance(t, ObjectT):
            flat = []
            for k, v in t.pairs:
                flat.extend([k, v])
            yield from self._eval_seq(flat, b, env, lambda vals: Obj(zip(vals[0::2], vals[1::2])))
            return
        if isinstance(t, ArrayCompr):
            out = []
            for b2 in self.eval_body(self._reordered(t.body, b, env), b, env):
                for v, _ in self.eval_term(t.term, b2, env):
                    out.append(v)
            yield Arr(out), b
            return
        if isinstance(t, SetCompr):
            out = RSet()
            for b2 in self.eval_body(self._reordered(t.body, b, env), b, env):
                for v, _ in self.eval_term(t.term, b2, env):
                    out.add(v)
            yield out, b
            return
        if isinstance(t, ObjectCompr):
            items = {}
            for b2 in self.eval_body(self._reordered(t.body, b, env), b, env):
                for k, b3 in self.eval_term(t.key, b2, env):
                    for v, _ in self.eval_term(t.value, b3, env):
                        if k in items and not rego_equal(items[k], v):
                            raise ConflictError("object keys must be unique")
                        items[k] = v
            yield Obj(items.items()), b
            return
        raise NotImplementedError(type(t))

    def _eval_seq(self, items, b, env, build, acc=()):
        if not items:
            yield build(list(acc)), b
            return
        for v, b2 in self.eval_term(items[0], b, env):
            yield from self._eval_seq(items[1:], b2, env, build, acc + (v,))

    def _eval_ref_head(self, name, path, i, b, env):
        if name == "input":
            if env.ctx.input is _UNDEF:
                return
            yield from self.walk_value(env.ctx.input, path, i, b, env)
            return
        if name == "data":
            yield from self.walk_data(self.root, env.ctx.data, path, i, b, env)
            return
        node = self._pkg_node(env.pkg)
        if node is not None and name in node.rules:
            pkg_path = [Scalar(p) for p in env.pkg] + [Scalar(name)]
            yield from self.walk_data(self.root, env.ctx.data, pkg_path + list(path), 0, b, env)
            return
        if env.module is not None:
            for ipath, alias in env.module.imports:
                if alias == name:
                    if ipath[0] == "input":
                        yield from self._eval_ref_head("input", [Scalar(p) for p in ipath[1:]] + list(path), 0, b, env)
                    else:
                        yield from self.walk_data(self.root, env.ctx.data, [Scalar(p) for p in ipath[1:]] + list(path), 0, b, env)
                    return
        raise RegoError("unsafe/undefined variable %s" % name)

    def walk_value(self, val, path, i, b, env):
        if i == len(path):
            yield val, b
            return
        sel = path[i]
        if self._is_unbound_var(sel, b, env):
            name = sel.name
            if isinstance(val, Obj):
                for k, v in list(val.items()):
                    b2 = dict(b)
                    b2[name] = k
                    yield from self.walk_value(v, path, i + 1, b2, env)
            elif isinstance(val, Arr):
                for idx, v in enumerate(val):
                    b2 = dict(b)
                    b2[name] = Num(str(idx))
                    yield from self.walk_value(v, path, i + 1, b2, env)
            elif isinstance(val, RSet):
                for v in list(val):
                    b2 = dict(b)
                    b2[name] = v
                    yield from self.walk_value(v, path, i + 1, b2, env)
            return
        if isinstance(sel, (ArrayT, ObjectT)) and not self._ground(sel, b, env):
            # pattern selector: iterate members and unify
            if isinstance(val, RSet):
                items = [(x, x) for x in val]
            elif isinstance(val, Obj):
                items = list(val.items())
            elif isinstance(val, Arr):
                items = [(Num(str(j)), x) for j, x in enumerate(val)]
            else:
                return
            for k, v in items:
                for b2 in self.unify_value(sel, k, b, env):
                    yield from self.walk_value(v, path, i + 1, b2, env)
            return
        for k, b2 in self.eval_term(sel, b, env):
            nv = _index(val, k)
            if nv is not _UNDEF:
                yield from self.walk_value(nv, path, i + 1, b2, env)

    def walk_data(self, node, base, path, i, b, env):
        if node is None or (not node.children and not node.rules):
            if base is _UNDEF or base is None:
                return
            yield from self.walk_value(base, path, i, b, env)
            return
        if i == len(path):
            yield self._materialize(node, base, env), b
            return
        sel = path[i]
        if self._is_unbound_var(sel, b, env):
            keys = list(node.children.keys()) + list(node.rules.keys())
            if isinstance(base, Obj):
                keys += [k for k in base.keys() if k not in node.children and k not in node.rules]
            for k in keys:
                b2 = dict(b)
                b2[sel.name] = k
                yield from self.walk_data(node, base, path[:i] + [Scalar(k)] + path[i + 1:], i, b2, env)
            return
        for k, b2 in self.eval_term(sel, b, env):
            if isinstance(k, str) and k in node.rules:
                yield from self.eval_rule_ref(node.rules[k], path, i + 1, b2, env)
            elif isinstance(k, str) and k in node.children:
                nb = base.get(k, _UNDEF) if isinstance(base, Obj) else _UNDEF
                yield from self.walk_data(node.children[k], nb, path, i + 1, b2, env)
            else:
                nb = _index(base, k) if base is not _UNDEF else _UNDEF
                if nb is not _UNDEF:
                    yield from self.walk_value(nb, path, i + 1, b2, env)

    def _materialize(self, node, base, env):
        items = list(base.items()) if isinstance(base, Obj) else []
        d = dict(items)
        for k, child in node.children.items():
            d[k] = self._materialize(child, d.get(k, _UNDEF), env)
        for name, rules in node.rules.items():
            if rules[0].kind == "func":
                continue
            vals = list(self.eval_rule_ref(rules, [], 0, {}, Env(env.ctx, rules[0].package, rules[0].module)))
            if vals:
                d[name] = vals[0][0]
        return Obj(d.items())

    # ------------------------------------------------------------------
    # virtual documents
    # ------------------------------------------------------------------
    def eval_rule_ref(self, rules, path, i, b, env):
        kind = rules[0].kind
        renv = Env(env.ctx, rules[0].package, rules[0].module)
        if kind == "complete":
            val = self._complete_value(rules, renv)
            if val is not _UNDEF:
                yield from self.walk_value(val, path, i, b, env)
            return
        if kind == "partial_set":
            if i == len(path):
                yield self._full_set(rules, renv), b
                return
            key_t = path[i]
            for r in rules:
                cb = self._prebind(r.key, key_t, b, env)
                if cb is None:
                    continue
                for sb in self.eval_body(self._rule_body(r, cb), cb, renv):
                    for kv, _ in self.eval_term(r.key, sb, renv):
                        for b2 in self.unify_value(key_t, kv, b, env):
                            yield from self.walk_value(kv, path, i + 1, b2, env)
            return
        if kind == "partial_obj":
            if i == len(path):
                yield self._full_obj(rules, renv), b
                return
            key_t = path[i]
            for r in rules:
                cb = self._prebind(r.key, key_t, b, env)
                if cb is None:
                    continue
                for sb in self.eval_body(self._rule_body(r, cb), cb, renv):
                    for kv, sb2 in self.eval_term(r.key, sb, renv):
                        for vv, _ in self.eval_term(r.value, sb2, renv):
                            for b2 in self.unify_value(key_t, kv, b, env):
                                yield from self.walk_value(vv, path, i + 1, b2, env)
            return
        raise RegoError("function %s referenced without call" % rules[0].name)

    def _prebind(self, head_t, caller_t, b, env):
        """Bind rule-head variables from ground parts of the caller's key term."""
        cb = {}
        if isinstance(head_t, Var) and self._ground(caller_t, b, env) and not isinstance(caller_t, Var):
            vals = list(self.eval_term(caller_t, b, env))
            if vals:
                cb[head_t.name] = vals[0][0]
            return cb
        if isinstance(caller_t, Var) and caller_t.name in b and isinstance(head_t, Var):
            cb[head_t.name] = b[caller_t.name]
            return cb
        if isinstance(head_t, ObjectT) and isinstance(caller_t, ObjectT):
            hk = {}
            for kt, vt in head_t.pairs:
                if isinstance(kt, Scalar):
                    hk[_hkey(kt.value)] = vt
            for kt, vt in caller_t.pairs:
                if isinstance(kt, Scalar) and _hkey(kt.value) in hk:
                    ht = hk[_hkey(kt.value)]
                    if isinstance(ht, Var) and self._ground(vt, b, env):
                        vals = list(self.eval_term(vt, b, env))
                        if vals:
                            cb[ht.name] = vals[0][0]
        return cb

    def _complete_value(self, rules, env):
        key = ("complete", id(rules[0]))
        cache = env.ctx.cache
        if key in cache:
            return cache[key]
        val = _UNDEF
        default = _UNDEF
        chain_rules = [r for r in rules if not r.default]
        for r in rules:
            if r.default:
                default = next(self.eval_term(r.value, {}, env))[0]
        # group else chains: a primary rule followed by its else rules
        groups = []
        for r in chain_rules:
            if r.is_else and groups:
                groups[-1].append(r)
            else:
                groups.append([r])
        for g in groups:
            for r in g:
                got = _UNDEF
                for sb in self.eval_body(self._rule_body(r, {}), {}, env):
                    for v, _ in self.eval_term(r.value, sb, env):
                        if got is not _UNDEF and not rego_equal(got, v):
                            raise ConflictError("complete rules must not produce multiple outputs")
                        got = v
                if got is not _UNDEF:
                    if val is not _UNDEF and not rego_equal(val, got):
                        raise ConflictError("complete rules must not produce multiple outputs")
                    val = got
                    break
        if val is _UNDEF:
            val = default
        cache[key] = val
        return val

    def _full_set(self, rules, env):
        key = ("set", id(rules[0]))
        cache = env.ctx.cache
        if key in cache:
            return cache[key]
        out = RSet()
        for r in rules:
            for sb in self.eval_body(self._rule_body(r, {}), {}, env):
                for v, _ in self.eval_term(r.key, sb, env):
                    out.add(v)
        cache[key] = out
        return out

    def _full_obj(self, rules, env):
        key = ("obj", id(rules[0]))
        cache = env.ctx.cache
        if key in cache:
            return cache[key]
        items = {}
        for r in rules:
            for sb in self.eval_body(self._rule_body(r, {}), {}, env):
                for k, sb2 in self.eval_term(r.key, sb, env):
                    for v, _ in self.eval_term(r.value, sb2, env):
                        if k in items and not rego_equal(items[k], v):
                            raise ConflictError("object keys must be unique")
                        items[k] = v
        out = Obj(items.items())
        cache[key] = out
        return out

    # ------------------------------------------------------------------
    # calls
    # ------------------------------------------------------------------
    def _resolve_func(self, op, env):
        if len(op) == 1:
            node = self._pkg_node(env.pkg)
            if node is not None and op[0] in node.rules:
                return node.rules[op[0]]
            if env.module is not None:
                for ipath, alias in env.module.imports:
                    if alias == op[0] and ipath[0] == "data":
                        n = self._pkg_node(tuple(ipath[1:-1]))
                        if n is not None and ipath[-1] in n.rules:
                            return n.rules[ipath[-1]]
            return None
        if op[0] == "data":
            n = self._pkg_node(tuple(op[1:-1]))
            if n is not None and op[-1] in n.rules:
                return n.rules[op[-1]]
            return None
        if env.module is not None:
            for ipath, alias in env.module.imports:
                if alias == op[0] and ipath[0] == "data":
                    full = list(ipath[1:]) + list(op[1:])
                    n = self._pkg_node(tuple(full[:-1]))
                    if n is not None and full[-1] in n.rules:
                        return n.rules[full[-1]]
        return None

    def eval_call(self, call: Call, b, env, statement=False):
        rules = self._resolve_func(call.op, env)
        name = ".".join(call.op)
        if rules is None:
            fn = B.BUILTINS.get(name)
            if fn is None:
                raise NotImplementedError("builtin %s" % name)
            arity = B.ARITY.get(name)
            args = call.args
            out_t = None
            if arity is not None and len(args) == arity + 1:
                args, out_t = args[:-1], args[-1]
            for vals, b2 in self._eval_args(args, b, env):
                v = fn(*vals)
                if v is _UNDEF or v is None:
                    continue
                if out_t is not None:
                    for b3 in self.unify_value(out_t, v, b2, env):
                        yield True, b3
                else:
                    yield v, b2
            return
        nargs = len(rules[0].args)
        args = call.args
        out_t = None
        if len(args) == nargs + 1:
            args, out_t = args[:-1], args[-1]
            statement = False
        for vals, b2 in self._eval_args(args, b, env):
            for v in self._call_func(rules, vals, statement and out_t is None, env.ctx):
                if self.call_hook is not None:
                    self.call_hook(rules[0], vals, v, env)
                if out_t is not None:
                    for b3 in self.unify_value(out_t, v, b2, env):
                        yield True, b3
                else:
                    yield v, b2

    def _eval_args(self, args, b, env, acc=()):
        if not args:
            yield list(acc), b
            return
        for v, b2 in self.eval_term(args[0], b, env):
            yield from self._eval_args(args[1:], b2, env, acc + (v,))

    def _call_func(self, rules, vals, statement, ctx):
        prev = _UNDEF
        for r in rules:
            env = Env(ctx, r.package, r.module)
            for cb in self._unify_args(r.args, vals, {}, env):
                for sb in self.eval_body(self._rule_body(r, cb), cb, env):
                    res = next(iter(self.eval_term(r.value, sb, env)), (_UNDEF, None))[0]
                    if res is _UNDEF:
                        continue
                    if statement and res is False:
                        continue
                    if prev is not _UNDEF:
                        if not rego_equal(prev, res):
                            raise ConflictError("functions must not produce multiple outputs for same inputs")
                        continue
                    prev = res
                    yield res

    def _unify_args(self, pats, vals, cb, env):
        if not pats:
            yield cb
            return
        for cb2 in self.unify_value(pats[0], vals[0], cb, env):
            yield from self._unify_args(pats[1:], vals[1:], cb2, env)

    # ------------------------------------------------------------------
    # safety reordering (ast/compiler.go reorderBodyForSafety, simplified)
    # ------------------------------------------------------------------
    def _rule_body(self, r: Rule, cb):
        key = ("rule", id(r), frozenset(cb.keys()))
        got = self._reorder_cache.get(key)
        if got is None:
            env = Env(None, r.package, r.module)
            safe = set(cb.keys())
            if r.args:
                for a in r.args:
                    safe |= set(_term_vars(a))
            body = expand_body(r.body)
            body = self._reorder(body, safe, env)
            got = rewrite_dynamics(body, lambda n: self._is_global(n, env))
            self._reorder_cache[key] = got
        return got

    def _reordered(self, body, b, env):
        # comprehension bodies are compiled together with their rule body
        return body

    def _reorder_nested_expr(self, e, safe, env):
        terms = [self._reorder_nested(t, safe, env) for t in e.terms]
        return Expr(e.kind, terms, negated=e.negated, withs=e.withs, loc=e.loc)

    def _reorder_nested(self, t, safe, env):
        if isinstance(t, ArrayCompr):
            return ArrayCompr(self._reorder_nested(t.term, safe, env), self._reorder(t.body, safe, env))
        if isinstance(t, SetCompr):
            return SetCompr(self._reorder_nested(t.term, safe, env), self._reorder(t.body, safe, env))
        if isinstance(t, ObjectCompr):
            return ObjectCompr(t.key, t.value, self._reorder(t.body, safe, env))
        if isinstance(t, Ref):
            return Ref(self._reorder_nested(t.head, safe, env), [self._reorder_nested(p, safe, env) for p in t.path])
        if isinstance(t, Call):
            return Call(t.op, [self._reorder_nested(a, safe, env) for a in t.args])
        if isinstance(t, ArrayT):
            return ArrayT([self._reorder_nested(x, safe, env) for x in t.items])
        if isinstance(t, SetT):
            return SetT([self._reorder_nested(x, safe, env) for x in t.items])
        if isinstance(t, ObjectT):
            return ObjectT([(self._reorder_nested(k, safe, env), self._reorder_nested(v, safe, env)) for k, v in t.pairs])
        return t

    def _reorder(self, body, safe, env):
        safe = set(safe)
        remaining = list(body)
        out = []
        globals_ = lambda n: self._is_global(n, env)
        while remaining:
            placed = False
            for e in remaining:
                needs, outs = _expr_needs_outputs(e, safe, globals_)
                if needs <= safe:
                    remaining.remove(e)
                    out.append(self._reorder_nested_expr(e, safe, env))
                    safe |= outs
                    placed = True
                    break
            if not placed:
                # leave the rest in order (unsafe bodies raise at eval time)
                out.extend(remaining)
                break
        return out


def _hkey(v):
    return ("k", v) if not isinstance(v, bool) else ("b", v)


def _index(val, k):
    if isinstance(val, Obj):
        if k in val:
            return val.get(k)
        return _UNDEF
    if isinstance(val, Arr):
        if isinstance(k, Num) and k.int64 is not None and 0 <= k.int64 < len(val):
            return val[k.int64]
        return _UNDEF
    if isinstance(val, RSet):
        if k in val:
            return k
        return _UNDEF
    return _UNDEF


# --------------------------------------------------------------------------
# variable analysis
# --------------------------------------------------------------------------


def _term_vars(t, out=None, skip_compr=True):
    if out is None:
        out = []
    if isinstance(t, Var):
        out.append(t.name)
    elif isinstance(t, Ref):
        _term_vars(t.head, out)
        for p in t.path:
            _term_vars(p, out)
    elif isinstance(t, Call):
        for a in t.args:
            _term_vars(a, out)
    elif isinstance(t, (ArrayT, SetT)):
        for x in t.items:
            _term_vars(x, out)
    elif isinstance(t, ObjectT):
        for k, v in t.pairs:
            _term_vars(k, out)
            _term_vars(v, out)
    elif isinstance(t, (ArrayCompr, SetCompr, ObjectCompr)):
        if not skip_compr:
            pass
    return out


def _compr_free_vars(t):
    """Variables a comprehension reads from its enclosing scope (approximate:
    vars used in its term/body that it never binds itself)."""
    body_vars = []
    bound = set()
    terms = []
    if isinstance(t, (ArrayCompr, SetCompr)):
        terms = [t.term]
    else:
        terms = [t.key, t.value]
    for e in t.body:
        for x in e.terms:
            body_vars += _all_vars(x)
        if e.kind in ("assign", "unify"):
            bound |= set(_all_vars(e.terms[0]))
            if e.kind == "unify":
                bound |= set(_all_vars(e.terms[1]))
        for x in e.terms:
            bound |= set(_iter_vars(x))
    return [v for v in body_vars + sum((_all_vars(x) for x in terms), []) if v not in bound and not v.startswith("$_")]


def _all_vars(t):
    out = []
    if isinstance(t, (ArrayCompr, SetCompr, ObjectCompr)):
        return _compr_free_vars(t)
    if isinstance(t, Var):
        out.append(t.name)
    elif isinstance(t, Ref):
        out += _all_vars(t.head)
        for p in t.path:
            out += _all_vars(p)
    elif isinstance(t, Call):
        for a in t.args:
            out += _all_vars(a)
    elif isinstance(t, (ArrayT, SetT)):
        for x in t.items:
            out += _all_vars(x)
    elif isinstance(t, ObjectT):
        for k, v in t.pairs:
            out += _all_vars(k) + _all_vars(v)
    return out


def _iter_vars(t):
    """Variables appearing directly as ref selectors (bound by iteration)."""
    out = []
    if isinstance(t, Ref):
        out += _iter_vars(t.head)
        for p in t.path:
            if isinstance(p, Var):
                out.append(p.name)
            else:
                out += _iter_vars(p)
    elif isinstance(t, Call):
        for a in t.args:
            out += _iter_vars(a)
    elif isinstance(t, (ArrayT, SetT)):
        for x in t.items:
            out += _iter_vars(x)
    elif isinstance(t, ObjectT):
        for k, v in t.pairs:
            out += _iter_vars(k) + _iter_vars(v)
    return out


def _expr_needs_outputs(e: Expr, safe, is_global):
    def vs(t):
        return {v for v in _all_vars(t) if not is_global(v)}

    def its(t):
        return {v for v in _iter_vars(t) if not is_global(v)}

    wvars = set()
    for w in e.withs:
        wvars |= vs(w.value)
    if e.kind == "some":
        return set(), set()
    if e.negated:
        needs = set()
        for t in e.terms:
            needs |= vs(t) - its(t)
        needs = {v for v in needs if not v.startswith("$_")}
        return needs | wvars, set()
    if e.kind == "term":
        t = e.terms[0]
        it = its(t) - safe
        needs, outs = (vs(t) - it), set(it)
        # hoisted call with a generated output variable (RewriteExprTerms)
        if isinstance(t, Call) and t.args and isinstance(t.args[-1], Var) and t.args[-1].name.startswith("$l") \
                and t.args[-1].name not in safe:
            needs.discard(t.args[-1].name)
            outs.add(t.args[-1].name)
        return needs | wvars, outs
    l, r = e.terms
    rn = vs(r) - its(r)
    if rn - safe == set():
        return rn | wvars | (its(r) & safe), vs(l) | its(r)
    if e.kind == "unify":
        ln = vs(l) - its(l)
        if ln - safe == set():
            return ln | wvars, vs(r) | its(l)
    return rn | wvars, set()


