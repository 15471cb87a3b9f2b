"""hooks.audit over the synced inventory (Client.Audit, client.go:805-833) as a
staged, device-resident batch (engine.cc audit_from_cache): the review of
each synced object is make_review / add_field's document
(target_template_source.go:46-89), built once per engine state.

CPU: the from-cache batch run by the CPU checker (oracle/cpuvm.cc) against
the oracle's own hooks.audit, with edge objects -- a JSON null (add_field
puts the namespace string in its place), a JSON false (dropped), an escaped
group/version, a group/version with two slashes (no review).  GPU: rows equal
the oracle's, and repeated audits reuse the batch until a mutation."""
import json

import pytest

import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, TARGET, data_path

from parity import oracle_for

AUDIT = 'hooks["%s"].audit' % TARGET


def _inventory(n_pods, seed):
    pods, ns_of, ns_objs = W.gen_pods(n_pods, seed=seed, n_namespaces=12)
    items = [(data_path(o), o) for o in list(ns_objs.values()) + pods]
    base = "/external/%s/namespace/team-0001" % TARGET
    items += [
        (base + "/v1/Pod/null-pod", None),                       # add_field: object := namespace
        (base + "/v1/Pod/false-pod", False),                     # add_field drops a falsy member
        (base + "/apps%2Fv1/Deployment/dep", {"apiVersion": "apps/v1", "kind": "Deployment",
                                              "metadata": {"name": "dep", "namespace": "team-0001"},
                                              "spec": {"template": {"spec": {"containers": []}}}}),
        (base + "/a%2Fb%2Fv1/Pod/two-slashes", pods[0]),         # make_group_version fails: no review
        ("/external/%s/cluster/v1/ConfigMap/cm" % TARGET, {"apiVersion": "v1", "kind": "ConfigMap",
                                                           "metadata": {"name": "cm"}}),
    ]
    return items


def _oracle_rows(od):
    return list(od.query(AUDIT))


def test_cache_batch_checker_equals_the_oracle_audit():
    from oracle import cpu_baseline
    ts, cs = W.config2()
    items = _inventory(200, 31)
    d = gkgpu.Driver(host_only=True)
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    od = oracle_for(ts, cs)
    for p, o in items:
        d.put_data(p, o)
        od.put_data(p, json.dumps(o))
    b = d.debug_stage_cache()
    assert b.n == len(items) - 1  # the two-slash group/version names no review
    evals, viol, flagged, digest = cpu_baseline.sweep_digest(d, b, threads=4)
    # the null object's review (object: a string) goes to the CPU driver for
    # its five constraints (ReviewCol fallback); nothing else is flagged
    assert flagged in (0, len(cs)), flagged
    want = _oracle_rows(od)
    assert viol == len(want) > 100, (viol, len(want))
    # row by row: the review's position in inventory path order, the engine's
    # constraint index, message and details (an order-free digest)
    import urllib.parse
    from oracle.driver import details_json
    order = {p: i for i, p in enumerate(sorted(p for p, _ in items if "%2Fb%2F" not in p))}
    cidx = {kn: i for i, kn in enumerate(d.constraints())}
    rows = []
    for r in want:
        rv, c = r["review"], r["constraint"]
        k = rv.get("kind")
        gv = k.get("version") if not k.get("group") else "%s/%s" % (k.get("group"), k.get("version"))
        ns = rv.get("namespace") if hasattr(rv, "get") else None
        path = ("/external/%s/namespace/%s/%s/%s/%s" % (TARGET, ns, urllib.parse.quote(gv, safe=""), k.get("kind"),
                                                         rv.get("name")) if isinstance(ns, str) else
                "/external/%s/cluster/%s/%s/%s" % (TARGET, urllib.parse.quote(gv, safe=""), k.get("kind"), rv.get("name")))
        rows.append((order[path], cidx[(c.get("kind"), c.get("metadata").get("name"))], r["msg"],
                     details_json(r["details"])))
    assert digest == cpu_baseline.row_digest(rows)


@pytest.mark.gpu
def test_audit_from_cache_reuses_the_staged_batch():
    """2,000 synced Pods + their Namespaces + the edge objects: Client.Audit's
    rows equal the oracle's (multiset of (kind, namespace, name, constraint,
    msg, details, action)); a second audit reuses the device batch; a put of
    a new object rebuilds it and the rows follow."""
    from oracle.driver import details_json
    ts, cs = W.config2()
    items = _inventory(2000, 32)
    drv = gkgpu.Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    od = oracle_for(ts, cs)
    for p, o in items:
        drv.put_data(p, o)
        od.put_data(p, json.dumps(o))

    def eng_rows():
        res = cl.audit()
        order = sorted(p for p, _ in items if "%2Fb%2F" not in p)
        # only the null object's review may go to the CPU driver
        assert all(order[i].endswith("/null-pod") for i, s in enumerate(res.status) if s), res.status
        out = []
        for r in res.results:
            seg = order[r.review].split("/")
            ns = seg[4] if seg[3] == "namespace" else ""
            out.append((seg[-2], ns, seg[-1], r.constraint_kind, r.constraint_name, r.msg, r.details_json,
                        r.enforcement_action))
        return sorted(out)

    def ref_rows():
        rows = []
        for r in _oracle_rows(od):
            rv, c = r["review"], r["constraint"]
            ns = rv.get("namespace") if hasattr(rv, "get") else None
            rows.append((rv.get("kind").get("kind"), ns if isinstance(ns, str) else "", rv.get("name"), c.get("kind"),
                         c.get("metadata").get("name"), r["msg"], details_json(r["details"]), r["enforcementAction"]))
        return sorted(rows)

    want = ref_rows()
    assert len(want) > 1000
    assert eng_rows() == want
    assert eng_rows() == want
    builds, reviews = drv.audit_cache_stats()
    assert builds == 1 and reviews == len(items) - 1, (builds, reviews)
    extra = W.gen_pods(1, seed=77, n_namespaces=12)[0][0]
    extra["metadata"]["name"] = "late-pod"
    p = data_path(extra)
    items.append((p, extra))
    drv.put_data(p, extra)
    od.put_data(p, json.dumps(extra))
    assert eng_rows() == ref_rows()
    assert drv.audit_cache_stats()[0] == 2


def _nssel_setup(n_pods, seed, host_only):
    """config 2 plus a container-limits constraint with a namespaceSelector,
    over Pods whose Namespaces are synced for only half of the namespaces.
    hooks.audit (regolib src.go:45-62) joins only matching_reviews_and_constraints:
    a Pod in an unsynced namespace fails matches_nsselector (get_ns has no
    solution, target_template_source.go:300-307) and yields no row -- in
    particular no autoreject "Namespace is not cached in OPA." row, which only
    hooks.violation emits (src.go:7-20)."""
    ts, cs = W.config2()
    cs = cs + [W.constraint("K8sContainerLimits", "dev-limits",
                            match={"kinds": [{"apiGroups": [""], "kinds": ["Pod"]}],
                                   "namespaceSelector": {"matchLabels": {"env": "dev"}}},
                            parameters={"cpu": "100m", "memory": "512Mi"})]
    pods, ns_of, ns_objs = W.gen_pods(n_pods, seed=seed, n_namespaces=12)
    synced = sorted(ns_objs)[::2]
    items = [(data_path(ns_objs[n]), ns_objs[n]) for n in synced] + [(data_path(o), o) for o in pods]
    d = gkgpu.Driver(host_only=host_only)
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    od = oracle_for(ts, cs)
    for p, o in items:
        d.put_data(p, o)
        od.put_data(p, json.dumps(o))
    return d, cl, od, cs, items, synced


def test_cache_audit_has_no_autoreject_rows_for_unsynced_namespaces():
    from oracle import cpu_baseline
    d, cl, od, cs, items, synced = _nssel_setup(240, 41, True)
    want = _oracle_rows(od)
    assert not any(r["msg"] == "Namespace is not cached in OPA." for r in want)
    assert any(r["constraint"].get("metadata").get("name") == "dev-limits" for r in want)
    b = d.debug_stage_cache()
    evals, viol, flagged, digest = cpu_baseline.sweep_digest(d, b, threads=4)
    assert flagged == 0
    assert viol == len(want), (viol, len(want))


@pytest.mark.gpu
def test_cache_audit_unsynced_namespace_under_namespace_selector():
    """GPU: the from-cache audit's rows equal the oracle's hooks.audit rows
    (no autoreject row) when half of the Pods' Namespaces are not synced."""
    from oracle.driver import details_json
    d, cl, od, cs, items, synced = _nssel_setup(1500, 42, False)
    order = sorted(p for p, _ in items)
    res = cl.audit()
    assert not any(res.status), "no review may be flagged"
    got = []
    for r in res.results:
        seg = order[r.review].split("/")
        ns = seg[4] if seg[3] == "namespace" else ""
        got.append((seg[-2], ns, seg[-1], r.constraint_kind, r.constraint_name, r.msg, r.details_json))
    want = []
    for r in _oracle_rows(od):
        rv, c = r["review"], r["constraint"]
        ns = rv.get("namespace")
        want.append((rv.get("kind").get("kind"), ns if isinstance(ns, str) else "", rv.get("name"), c.get("kind"),
                     c.get("metadata").get("name"), r["msg"], details_json(r["details"])))
    assert not any(w[5] == "Namespace is not cached in OPA." for w in want)
    assert sorted(got) == sorted(want)


@pytest.mark.gpu
def test_audit_cache_sample_totals_and_first_results():
    """gk_audit_cache_sample: the from-cache audit reduced on the device as
    the audit manager consumes it (manager.go:195-207, :462-508) -- exact
    per-constraint totals and the first 20 results per constraint in
    inventory order -- equal the oracle's hooks.audit rows counted and cut the
    same way; the staged batch is shared with gk_query(hooks.audit)."""
    import collections
    ts, cs = W.config2()
    items = _inventory(1500, 33)
    items = [(p, o) for p, o in items if not p.endswith("/null-pod")]  # no CPU-driver review
    drv = gkgpu.Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    od = oracle_for(ts, cs)
    for p, o in items:
        drv.put_data(p, o)
        od.put_data(p, json.dumps(o))
    order = sorted(p for p, _ in items if "%2Fb%2F" not in p)
    idx = {}
    for i, p in enumerate(order):
        seg = p.split("/")
        idx[(seg[-2], seg[4] if seg[3] == "namespace" else "", seg[-1])] = i
    cons = drv.constraints()
    cidx = {kn: i for i, kn in enumerate(cons)}
    per = collections.defaultdict(list)  # constraint -> [(review, k, msg)] in evaluation order
    for k, r in enumerate(_oracle_rows(od)):
        rv, c = r["review"], r["constraint"]
        ns = rv.get("namespace")
        key = (rv.get("kind").get("kind"), ns if isinstance(ns, str) else "", rv.get("name"))
        per[cidx[(c.get("kind"), c.get("metadata").get("name"))]].append((idx[key], k, r["msg"]))
    sw = drv.audit_sample(limit=20)
    assert not sw.flagged and sw.n_errors == 0 and sw.n_fallbacks == 0
    assert sw.totals == [len(per[c]) for c in range(len(cons))]
    got = collections.defaultdict(list)
    for s in sw.samples:
        got[s.constraint].append((s.review, s.msg.decode("utf-8", "surrogateescape")))
    for c in range(len(cons)):
        want = [(rv, m[:256]) for rv, _k, m in sorted(per[c])[:20]]
        assert got[c] == want, (cons[c], got[c][:3], want[:3])
    # one staged batch for both entry points
    assert drv.audit_summary()["results"] == sum(sw.totals)
    assert drv.audit_cache_stats()[0] == 1
