"""Oracle implementation of the frameworks ``drivers.Driver`` for the K8s target.

Test infrastructure only.  Restates what the reference's local OPA driver
computes for the two hot-path queries:

* ``hooks["admission.k8s.gatekeeper.sh"].violation`` with ``{"review": ...}``
  (per-object audit / webhook; ``client.go:763-800``, hooks ``regolib/src.go:23-43``);
* ``hooks["admission.k8s.gatekeeper.sh"].audit`` over the synced inventory
  (``client.go:805-833``, ``regolib/src.go:45-61``,
  ``target_template_source.go:46-89``).

The match library and hooks are Python (``oracle.match``); ConstraintTemplate
Rego is interpreted by ``oracle.rego``.  Storage paths follow
``drivers/local/local.go`` (``PutData`` / ``DeleteData`` on ``/``-separated,
URL-unescaped paths; ``storage/path.go:35-47``).
"""
from __future__ import annotations

import re
import urllib.parse

from . import match as M
from .rego import Interpreter, parse_module
from .rego.values import NULL, Arr, Obj, RegoError, RSet, from_json_text, go_json_marshal, rego_equal

TARGET = "admission.k8s.gatekeeper.sh"
CONSTRAINT_GROUP = "constraints.gatekeeper.sh"


class QueryError(Exception):
    pass


def _parse_path(p: str):
    parts = [x for x in p.strip("/").split("/") if x != ""]
    return [urllib.parse.unquote(x) for x in parts]


def _obj_set(root, path, value):
    if not path:
        return value
    k = path[0]
    child = root.get(k) if isinstance(root, Obj) and k in root else Obj()
    base = root if isinstance(root, Obj) else Obj()
    return base.with_item(k, _obj_set(child, path[1:], value))


def _obj_del(root, path):
    if not isinstance(root, Obj) or path[0] not in root:
        return root, False
    if len(path) == 1:
        o = Obj((k, v) for k, v in root.items() if k != path[0])
        return o, True
    child, ok = _obj_del(root.get(path[0]), path[1:])
    if not ok:
        return root, False
    return root.with_item(path[0], child), True


def _pkg_of(name: str):
    """`templates["t"]["K"]` -> ('templates','t','K')."""
    out = []
    for m in re.finditer(r'([A-Za-z_][A-Za-z0-9_]*)|\["((?:[^"\\]|\\.)*)"\]', name):
        out.append(m.group(1) if m.group(1) is not None else m.group(2))
    return tuple(out)


class OracleDriver:
    """drivers.Driver restatement (interface.go:21-39) for the K8s target."""

    def __init__(self):
        self.modules = {}  # name -> source
        self.data = Obj()
        self.interp = Interpreter()
        self._dirty = True

    # -- modules ------------------------------------------------------------
    def put_module(self, name, src):
        self.modules[name] = src
        self._dirty = True

    def put_modules(self, prefix, srcs):
        self.delete_modules(prefix)
        for i, s in enumerate(srcs):
            self.modules["__modset_%s_idx_%d" % (prefix, i)] = s
        self._dirty = True

    def delete_module(self, name):
        ok = self.modules.pop(name, None) is not None
        self._dirty = True
        return ok

    def delete_modules(self, prefix):
        keys = [k for k in self.modules if k.startswith("__modset_%s_idx_" % prefix)]
        for k in keys:
            del self.modules[k]
        self._dirty = True
        return len(keys)

    def _rebuild(self):
        if not self._dirty:
            return
        it = Interpreter()
        for name, src in self.modules.items():
            m = parse_module(src)
            # the hooks/library modules are restated natively (oracle.match)
            if m.package[:1] == ("hooks",):
                continue
            it.add_module(m)
        self.interp = it
        self._dirty = False

    # -- data ---------------------------------------------------------------
    def put_data(self, path, value):
        if isinstance(value, str):
            value = from_json_text(value)
        self.data = _obj_set(self.data, _parse_path(path), value)

    def delete_data(self, path):
        p = _parse_path(path)
        if not p:
            self.data = Obj()
            return True
        self.data, ok = _obj_del(self.data, p)
        return ok

    # -- views --------------------------------------------------------------
    def constraints_root(self):
        return M.path(self.data, "constraints", TARGET, "cluster", CONSTRAINT_GROUP)

    def external(self):
        return M.path(self.data, "external", TARGET)

    def ns_cache(self):
        return M.path(self.data, "external", TARGET, "cluster", "v1", "Namespace")

    # -- template evaluation ------------------------------------------------
    def template_violations(self, kind, inp, inv):
        """data.templates[T][kind].violation[r] with input as inp with data.inventory as inv."""
        self._rebuild()
        it = self.interp
        node = it._pkg_node(("templates", TARGET, kind))
        if node is None or "violation" not in node.rules:
            return []
        saved = it.data
        it.data = self.data.with_item("inventory", inv)
        try:
            return it.query_ref(("templates", TARGET, kind, "violation"), inp)
        finally:
            it.data = saved

    # -- queries ------------------------------------------------------------
    def query(self, path, input_val=None):
        """Returns a list of result dicts (msg, details, constraint, review,
        enforcementAction) in evaluation order, or raises QueryError."""
        if isinstance(input_val, str):
            input_val = from_json_text(input_val)
        try:
            if path == 'hooks["%s"].violation' % TARGET:
                return self._violation(input_val)
            if path == 'hooks["%s"].audit' % TARGET:
                return self._audit()
        except RegoError as e:
            raise QueryError(str(e))
        raise NotImplementedError(path)

    def _inventory(self):
        ext = self.external()
        return ext if M.truthy(ext) else Obj()

    def _responses(self, review, constraint):
        out = []
        params = _hget(_hget(constraint, "spec", Obj()), "parameters", Obj())
        inp = Obj([("review", review), ("parameters", params)])
        kind = M.index(constraint, "kind")
        if not isinstance(kind, str):
            return out
        for r in self.template_violations(kind, inp, self._inventory()):
            msg = M.index(r, "msg")
            if msg is M.UNDEF:
                continue
            details = _hget(r, "details", Obj())
            spec = _hget(constraint, "spec", Obj())
            ea = _hget(spec, "enforcementAction", "deny")
            out.append(_result(msg, details, constraint, review, ea))
        return out

    def _violation(self, input_val):
        review = _hget(input_val, "review", Obj())
        croot = self.constraints_root()
        nsc = self.ns_cache()
        out = []
        # rule 1: autoreject
        if input_val is not None and input_val is not M.UNDEF:
            rin = M.index(input_val, "review")
            for rej in M.autoreject_review(rin, croot, nsc):
                c = _hget(rej, "constraint", Obj())
                ea = _hget(_hget(c, "spec", Obj()), "enforcementAction", "deny")
                out.append(_result(_hget(rej, "msg", ""), _hget(rej, "details", Obj()), c, review, ea))
            # rule 2: matching constraints x template violations
            for c in M.matching_constraints(rin, croot, nsc):
                out.extend(self._responses(review, c))
        return out

    def _audit(self):
        croot = self.constraints_root()
        nsc = self.ns_cache()
        ext = self.external()
        out = []
        for review in _inventory_reviews(ext):
            for c in M.matching_constraints(review, croot, nsc):
                out.extend(self._responses(review, c))
        return out


def _inventory_reviews(ext):
    """matching_reviews_and_constraints review construction (:46-89)."""
    for ns, by_gv in M.items(M.index(ext, "namespace")):
        for gv, by_kind in M.items(by_gv):
            for kind, by_name in M.items(by_kind):
                for name, obj in M.items(by_name):
                    r = _make_review(obj, gv, kind, name)
                    if r is None:
                        continue
                    yield _add_field(r, "namespace", ns)
    for gv, by_kind in M.items(M.index(ext, "cluster")):
        for kind, by_name in M.items(by_kind):
            for name, obj in M.items(by_name):
                r = _make_review(obj, gv, kind, name)
                if r is not None:
                    yield r


def _make_review(obj, api_version, kind, name):
    gv = M.make_group_version(api_version)
    if gv is M.UNDEF:
        return None
    group, version = gv[0], gv[1]
    return Obj([("kind", Obj([("group", group), ("version", version), ("kind", kind)])), ("name", name),
                ("object", obj)])


def _add_field(obj, key, value):
    keys = [k for k, v in obj.items() if v is not False]
    all_keys = RSet(keys)
    all_keys.add(key)
    return Obj((k, M.get_default(obj, k, value)) for k in all_keys)


def _hget(obj, field, default):
    """Hooks-level get_default (regolib/src.go:77-85): obj[field] if defined (null kept)."""
    v = M.index(obj, field)
    return default if v is M.UNDEF else v


def _result(msg, details, constraint, review, ea):
    # local.go:341-352 JSON round trip into types.Result: non-string msg or
    # enforcementAction fail to unmarshal -> the Query errors.
    if not isinstance(msg, str):
        raise QueryError("json: cannot unmarshal into Result.msg")
    if ea is not NULL and not isinstance(ea, str):
        raise QueryError("json: cannot unmarshal into Result.enforcementAction")
    return {"msg": msg, "details": details, "constraint": constraint, "review": review,
            "enforcementAction": "" if ea is NULL else ea}


def details_json(details) -> str:
    return go_json_marshal(details)
