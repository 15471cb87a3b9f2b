"""Gatekeeper target match library, restated in Python — oracle only.

Follows ``pkg/target/target_template_source.go`` (the Rego library the
frameworks client installs as ``hooks["admission.k8s.gatekeeper.sh"].library``)
rule by rule, with OPA v0.21 evaluation semantics:

* functions yield at most once; evaluation order (and therefore which builtin
  errors are reachable) follows the Rego bodies;
* refs to ``input`` used as call arguments (and ref-valued selectors) are
  evaluated *before* a surrounding ``not`` (OPA RewriteDynamicTerms; pinned by
  ``pkg/target/regolib/autoreject_test.rego:test_with_undefined_ns``), while
  refs rooted at local variables stay inside it (pinned by
  ``util_test.rego:test_has_field_no_field`` and
  ``target_integration_test.go`` "match deny all").

Every function takes plain oracle values (``oracle.rego.values``) and returns a
value, ``True`` for a defined boolean-rule, or ``UNDEF``.  Builtin type errors
raise :class:`oracle.rego.values.RegoError`.
"""
from __future__ import annotations

from .rego import builtins as B
from .rego.values import NULL, Arr, Num, Obj, RegoError, RSet, rego_equal

UNDEF = object()


# --------------------------------------------------------------------------
# value helpers (Rego ref indexing / iteration)
# --------------------------------------------------------------------------


def index(v, k):
    if v is UNDEF:
        return UNDEF
    if isinstance(v, Obj):
        return v.get(k) if k in v else UNDEF
    if isinstance(v, Arr):
        if isinstance(k, Num) and k.int64 is not None and 0 <= k.int64 < len(v):
            return v[k.int64]
        return UNDEF
    if isinstance(v, RSet):
        return k if k in v else UNDEF
    return UNDEF


def path(v, *keys):
    for k in keys:
        v = index(v, k)
        if v is UNDEF:
            return UNDEF
    return v


def items(v):
    """(key, value) pairs that `v[k]` iteration visits."""
    if isinstance(v, Obj):
        return list(v.items())
    if isinstance(v, Arr):
        return [(Num(str(i)), x) for i, x in enumerate(v)]
    if isinstance(v, RSet):
        return [(x, x) for x in v]
    return []


def truthy(v):
    return v is not UNDEF and v is not False


def eq(a, b):
    return a is not UNDEF and b is not UNDEF and rego_equal(a, b)


EMPTY_OBJ = Obj()


# --------------------------------------------------------------------------
# util (target_template_source.go:91-125)
# --------------------------------------------------------------------------


def has_field(obj, field):
    """:91-105 — true when obj[field] is defined (incl. false); else false."""
    return index(obj, field) is not UNDEF


def get_default(obj, field, default):
    """:110-125 — obj[field] unless missing or null."""
    v = index(obj, field)
    if v is UNDEF or v is NULL:
        return default
    return v


def make_group_version(api_version):
    """:72-81."""
    if not isinstance(api_version, str):
        raise RegoError("operand 1 must be string")
    if "/" in api_version:
        parts = api_version.split("/")
        if len(parts) == 2:
            return Arr(parts)
        return UNDEF
    return Arr(["", api_version])


# --------------------------------------------------------------------------
# kind selector (:131-156)
# --------------------------------------------------------------------------


def any_kind_selector_matches(match, review):
    kind_selectors = get_default(match, "kinds", Arr([Obj([("apiGroups", Arr(["*"])), ("kinds", Arr(["*"]))])]))
    for _, ks in items(kind_selectors):
        if kind_selector_matches(ks, review):
            return True
    return UNDEF


def kind_selector_matches(ks, review):
    return group_matches(ks, review) and kind_matches(ks, review)


def group_matches(ks, review):
    groups = index(ks, "apiGroups")
    for _, g in items(groups):
        if eq(g, "*"):
            return True
    grp = path(review, "kind", "group")
    for _, g in items(groups):
        if eq(g, grp):
            return True
    return False


def kind_matches(ks, review):
    kinds = index(ks, "kinds")
    for _, k in items(kinds):
        if eq(k, "*"):
            return True
    kd = path(review, "kind", "kind")
    for _, k in items(kinds):
        if eq(k, kd):
            return True
    return False


# --------------------------------------------------------------------------
# scope (:162-178)
# --------------------------------------------------------------------------


def matches_scope(match, review):
    if not has_field(match, "scope"):
        return True
    sc = index(match, "scope")
    if eq(sc, "*"):
        return True
    if eq(sc, "Namespaced"):
        if review is not UNDEF and not rego_equal(get_default(review, "namespace", ""), ""):
            return True
    if eq(sc, "Cluster"):
        if review is not UNDEF and rego_equal(get_default(review, "namespace", ""), ""):
            return True
    return UNDEF


# --------------------------------------------------------------------------
# label selector (:185-281)
# --------------------------------------------------------------------------


def match_expression_violated(op, labels, key, values):
    """:185-213.  Evaluates every rule body (all can raise) and yields true once."""
    res = UNDEF
    if eq(op, "In"):
        if has_field(labels, key) is False:
            res = True
        if B.gt(B.count(values), Num("0")):
            value_set = RSet(v for _, v in items(values))
            lv = index(labels, key)
            if lv is not UNDEF and B.neq(B.count(B.minus(RSet([lv]), value_set)), Num("0")):
                res = True
    elif eq(op, "NotIn"):
        if B.gt(B.count(values), Num("0")):
            value_set = RSet(v for _, v in items(values))
            lv = index(labels, key)
            if lv is not UNDEF and B.equal(B.count(B.minus(RSet([lv]), value_set)), Num("0")):
                res = True
    elif eq(op, "Exists"):
        if has_field(labels, key) is False:
            res = True
    elif eq(op, "DoesNotExist"):
        if has_field(labels, key) is True:
            res = True
    return res


def matches_label_selector(selector, labels):
    """:218-230."""
    match_labels = get_default(selector, "matchLabels", EMPTY_OBJ)
    satisfied = RSet()
    for k, v in items(match_labels):
        lv = index(labels, k)
        if lv is not UNDEF and rego_equal(v, lv):
            satisfied.add(k)
    if not B.equal(B.count(satisfied), B.count(match_labels)):
        return UNDEF
    match_exprs = get_default(selector, "matchExpressions", Arr())
    mismatches = RSet()
    for _, me in items(match_exprs):
        values = get_default(me, "values", Arr())
        op = index(me, "operator")
        key = index(me, "key")
        if op is UNDEF or key is UNDEF:
            continue
        r = match_expression_violated(op, labels, key, values)
        if r is not UNDEF:
            mismatches.add(r)
    if B.any_(mismatches) is False:
        return True
    return UNDEF


def _labels_of(obj):
    return get_default(get_default(obj, "metadata", EMPTY_OBJ), "labels", EMPTY_OBJ)


def any_labelselector_match(label_selector, review):
    """:233-281 (object / oldObject combinations)."""
    if review is UNDEF:
        return UNDEF
    old = get_default(review, "oldObject", EMPTY_OBJ)
    obj = get_default(review, "object", EMPTY_OBJ)
    old_empty = rego_equal(old, EMPTY_OBJ)
    obj_empty = rego_equal(obj, EMPTY_OBJ)
    out = UNDEF
    if old_empty and not obj_empty:
        if matches_label_selector(label_selector, _labels_of(obj)) is True:
            out = True
    if not old_empty and obj_empty:
        if matches_label_selector(label_selector, _labels_of(old)) is True:
            out = True
    if not old_empty and not obj_empty:
        ms = RSet()
        for l in (_labels_of(obj), _labels_of(old)):
            r = matches_label_selector(label_selector, l)
            if r is not UNDEF:
                ms.add(r)
        if B.any_(ms):
            out = True
    if old_empty and obj_empty:
        if matches_label_selector(label_selector, EMPTY_OBJ) is True:
            out = True
    return out


# --------------------------------------------------------------------------
# namespace logic (:287-386)
# --------------------------------------------------------------------------


def is_ns(kind):
    return eq(index(kind, "group"), "") and eq(index(kind, "kind"), "Namespace")


def get_ns(review, ns_cache):
    """:292-299, partial set — list of solutions (no dedupe)."""
    out = []
    un = path(review, "_unstable", "namespace")
    if un is not UNDEF:
        out.append(un)
    if not truthy(un):
        nsname = index(review, "namespace")
        v = index(ns_cache, nsname) if nsname is not UNDEF else UNDEF
        if v is not UNDEF:
            out.append(v)
    return out


def get_ns_name(review):
    out = []
    kind = index(review, "kind")
    if kind is not UNDEF and is_ns(kind):
        n = path(review, "object", "metadata", "name")
        if n is not UNDEF:
            out.append(n)
    if kind is not UNDEF and not is_ns(kind):
        n = index(review, "namespace")
        if n is not UNDEF:
            out.append(n)
    return out


def always_match_ns_selectors(review):
    kind = index(review, "kind")
    if kind is UNDEF or is_ns(kind):
        return False
    return rego_equal(get_default(review, "namespace", ""), "")


def _ns_list_test(match, field, review, want_in):
    if not has_field(match, field):
        return True
    if always_match_ns_selectors(review):
        return True
    for ns in get_ns_name(review):
        nss = RSet(v for _, v in items(index(match, field)))
        c = B.count(B.minus(RSet([ns]), nss))
        if want_in and B.equal(c, Num("0")):
            return True
        if not want_in and B.neq(c, Num("0")):
            return True
    return UNDEF


def matches_namespaces(match, review):
    """:318-330."""
    return _ns_list_test(match, "namespaces", review, True)


def does_not_match_excludednamespaces(match, review):
    """:332-344."""
    return _ns_list_test(match, "excludedNamespaces", review, False)


def matches_namespace_selector(match, ns):
    """:380-386."""
    nslabels = get_default(get_default(ns, "metadata", EMPTY_OBJ), "labels", EMPTY_OBJ)
    sel = get_default(match, "namespaceSelector", EMPTY_OBJ)
    return matches_label_selector(sel, nslabels)


def matches_nsselector(match, review, ns_cache):
    """:346-376."""
    out = UNDEF
    if not has_field(match, "namespaceSelector"):
        out = True
    if has_field(match, "namespaceSelector") and always_match_ns_selectors(review):
        out = True
    kind = index(review, "kind")
    if kind is not UNDEF and not is_ns(kind) and not always_match_ns_selectors(review) \
            and has_field(match, "namespaceSelector"):
        for ns in get_ns(review, ns_cache):
            if matches_namespace_selector(match, ns) is True:
                out = True
    if kind is not UNDEF and is_ns(kind) and not always_match_ns_selectors(review) \
            and has_field(match, "namespaceSelector"):
        if any_labelselector_match(get_default(match, "namespaceSelector", EMPTY_OBJ), review) is True:
            out = True
    return out


# --------------------------------------------------------------------------
# top-level rules
# --------------------------------------------------------------------------


def constraint_matches(constraint, review, ns_cache):
    """Body of matching_constraints[constraint] (:27-44) for one constraint."""
    spec = get_default(constraint, "spec", EMPTY_OBJ)
    match = get_default(spec, "match", EMPTY_OBJ)
    if any_kind_selector_matches(match, review) is not True:
        return False
    if matches_namespaces(match, review) is not True:
        return False
    if does_not_match_excludednamespaces(match, review) is not True:
        return False
    if matches_nsselector(match, review, ns_cache) is not True:
        return False
    if matches_scope(match, review) is not True:
        return False
    label_selector = get_default(match, "labelSelector", EMPTY_OBJ)
    if any_labelselector_match(label_selector, review) is not True:
        return False
    return True


def iter_constraints(constraints_root):
    """data.constraints[T].cluster["constraints.gatekeeper.sh"][_][_] in storage order."""
    for _, by_kind in items(constraints_root):
        for _, c in items(by_kind):
            yield c


def matching_constraints(review, constraints_root, ns_cache):
    return [c for c in iter_constraints(constraints_root) if constraint_matches(c, review, ns_cache)]


def autoreject_review(review, constraints_root, ns_cache):
    """:12-25."""
    out = []
    for c in iter_constraints(constraints_root):
        spec = get_default(c, "spec", EMPTY_OBJ)
        match = get_default(spec, "match", EMPTY_OBJ)
        if not has_field(match, "namespaceSelector"):
            continue
        nsname = index(review, "namespace")
        if nsname is UNDEF:
            continue  # hoisted ref is undefined
        if truthy(index(ns_cache, nsname)):
            continue
        if truthy(path(review, "_unstable", "namespace")):
            continue
        if rego_equal(nsname, ""):
            continue
        out.append(Obj([("msg", "Namespace is not cached in OPA."), ("details", Obj()), ("constraint", c)]))
    return out
