"""Inventory joins as a device pass (compiler.cc join_site, engine.cc
build_joins, kernels.hip gk_key_kernel, devrt.h op_jprobe).

The reference scans the whole synced inventory per review
(k8suniqueserviceselector_template.yaml:40-44, k8suniquelabel_template.yaml:49-52;
SURVEY 8(f)3 asks for a hash-join pass).  The engine compiles such an
iteration as a probe of a per-constraint hash index whose keys a device key
pass computes per inventory leaf; the plain scan stays beside it for lanes
without an index.  CPU tests: which templates get join sites and which
shapes are refused.  GPU tests: the probe path against the oracle (edge
cases: failing key programs, numeric and composite keys, inventory changes)
and against the scan path (GKGPU_JOINS=0) at a few thousand objects.
"""
import collections
import json
import os

import pytest

import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, data_path

from parity import compare, engine_rows, oracle_for, run_objects
from gkgpu.client import augmented_review

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _driver(ts, cs, extra=(), **kw):
    d = gkgpu.Driver(**kw)
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    for p, o in extra:
        d.put_data(p, o)
    return d


def test_join_sites_of_the_cross_resource_templates():
    ts, cs = W.config6()
    d = _driver(ts, cs, host_only=True)
    assert d.template_joins("K8sUniqueServiceSelector") == ["data.inventory.namespace[_][_][_][_]"]
    # unique-label: both lazy inventory comprehensions (cluster, namespace scope)
    assert d.template_joins("K8sUniqueLabel") == ["data.inventory.cluster[_][_][_]",
                                                  "data.inventory.namespace[_][_][_][_]"]
    for k in ("K8sRequiredLabels", "K8sAllowedRepos", "K8sContainerLimits", "K8sRequiredProbes"):
        assert d.template_joins(k) == []
    # agilebank's dry-run unique-ingress-host: every rule host is a key value,
    # re_match over the apiVersion path variable is skipped outside the bucket
    d = _driver([W.UNIQUE_INGRESS_HOST], [W.constraint("K8sUniqueIngressHost", "u")], host_only=True)
    assert d.template_joins("K8sUniqueIngressHost") == ["data.inventory.namespace[_][_].Ingress[_]"]


def test_join_switch_off(monkeypatch):
    monkeypatch.setenv("GKGPU_JOINS", "0")
    ts, cs = W.config6()
    d = _driver(ts, cs, host_only=True)
    assert d.template_joins("K8sUniqueServiceSelector") == []
    assert d.template_joins("K8sUniqueLabel") == []


def _tmpl(kind, body):
    return W._tmpl(kind, "package %s\n\n%s" % (kind.lower(), body))


# a skipped literal that may raise (conflicting function values): no join
MAY_ERR = _tmpl("K8sJoinMayErr", """
pick(o) = v { v := o.metadata.name }
pick(o) = v { v := o.kind }

violation[{"msg": msg}] {
	val := input.review.object.metadata.labels.app
	other := data.inventory.namespace[ns][_][_][name]
	pick(other) != "x"
	val == other.metadata.labels.app
	msg := sprintf("dup %v/%v", [ns, name])
}
""")

# the key reads the review: not a function of the leaf alone, no join
KEY_READS_REVIEW = _tmpl("K8sJoinKeyReview", """
violation[{"msg": msg}] {
	val := input.review.object.metadata.labels.app
	other := data.inventory.namespace[ns][_][_][name]
	k := concat("/", [other.metadata.labels.app, input.review.object.kind])
	val == k
	msg := sprintf("dup %v/%v", [ns, name])
}
""")

# exclusive function bodies (== / != on one path) and a parameter-derived key
LABEL_PARAM = _tmpl("K8sJoinLabelParam", """
ver(k) = v { k.group != ""; v := sprintf("%v/%v", [k.group, k.version]) }
ver(k) = v { k.group == ""; v := k.version }

violation[{"msg": msg}] {
	label := input.parameters.label
	val := input.review.object.spec.tags[label]
	other := data.inventory.namespace[ns][_][kind][name]
	not other.apiVersion == ver(input.review.kind)
	val == other.spec.tags[label]
	msg := sprintf("%v %v/%v/%v has %v", [label, ns, kind, name, val])
}
""")


def test_join_planner_refuses_unsafe_shapes():
    cs = [W.constraint("K8sJoinMayErr", "a"), W.constraint("K8sJoinKeyReview", "b"),
          W.constraint("K8sJoinLabelParam", "c", parameters={"label": "app"})]
    d = _driver([MAY_ERR, KEY_READS_REVIEW, LABEL_PARAM], cs, host_only=True)
    assert d.template_status("K8sJoinMayErr")[0] == 1
    assert d.template_joins("K8sJoinMayErr") == []
    assert d.template_joins("K8sJoinKeyReview") == []
    assert d.template_joins("K8sJoinLabelParam") == ["data.inventory.namespace[_][_][_][_]"]


def _labelled(n, seed, value=lambda r, i: "v%d" % r.randint(0, 9)):
    import random
    r = random.Random(seed)
    out = []
    for i in range(n):
        tags = {"app": value(r, i)} if r.random() < 0.8 else {}
        kind, av = (("ConfigMap", "v1"), ("Deployment", "apps/v1"))[i % 2]
        out.append({"apiVersion": av, "kind": kind,
                    "metadata": {"name": "o-%04d" % i, "namespace": "ns-%d" % (i % 5)}, "spec": {"tags": tags}})
    return out


def _ns(objs):
    return [{"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": o["metadata"]["namespace"]}} for o in objs]


def _oracle_count(od, objs, nss):
    from parity import oracle_review
    n = 0
    for o, ns in zip(objs, nss):
        r = oracle_review(od, augmented_review(o, ns))
        assert r != "ERROR"
        n += len(r)
    return n


def test_checker_probe_equals_scan_and_oracle():
    """The probe code the compiler emits, run by the CPU checker with its own
    host-built indexes (oracle/cpuvm.cc gkcpu_build_joins), against the scan
    beside it and the oracle: tag values of every JSON type, and config 6."""
    from oracle import cpu_baseline
    vals = ["a", "b", 7, 7.0, True, None, {"x": 1}, "a", 3, False]
    objs = _labelled(120, 5, value=lambda r, i: vals[r.randint(0, len(vals) - 1)])
    cs = [W.constraint("K8sJoinLabelParam", "c", parameters={"label": "app"})]
    extra = [(data_path(o), o) for o in objs]
    d = _driver([LABEL_PARAM], cs, extra, host_only=True)
    b = d.stage_objects(objs, _ns(objs))
    probe = cpu_baseline.sweep(d, b, threads=2)[1:]
    scan = cpu_baseline.sweep(d, b, threads=2, joins=False)[1:]
    assert probe == scan and probe[3] == 0, (probe, scan)
    assert probe[1] == _oracle_count(oracle_for([LABEL_PARAM], cs, extra), objs, _ns(objs)) > 100
    ts, cs = W.config6()
    objs_js, nss_js = W.gen_config6_json(1200)
    inv = [(p, json.loads(o)) for p, o in W.inventory_paths(objs_js)]
    d = _driver(ts, cs, inv, host_only=True)
    b = d.stage_objects(objs_js, nss_js)
    probe = cpu_baseline.sweep(d, b, threads=4)
    scan = cpu_baseline.sweep(d, b, threads=4, joins=False)
    assert probe[1:] == scan[1:] and probe[4] == 0 and probe[2] > 500, (probe, scan)


def test_checker_multi_valued_keys_and_array_levels():
    """unique-ingress-host (1-3 hosts per Ingress, colliding; a rule without a
    host; an apiVersion outside the regex): checker probe = scan = oracle.
    Then an array synced where a path variable iterates (its key would be an
    index, not a string, and re_match would fail): the site is left to the
    scan, which fails those reviews exactly as before."""
    from oracle import cpu_baseline
    objs, nss = W.gen_ingresses(300)
    cs = [W.constraint("K8sUniqueIngressHost", "uih")]
    extra = [(data_path(o), o) for o in objs]
    d = _driver([W.UNIQUE_INGRESS_HOST], cs, extra, host_only=True)
    b = d.stage_objects(objs, nss)
    probe = cpu_baseline.sweep(d, b, threads=4)[1:]
    scan = cpu_baseline.sweep(d, b, threads=4, joins=False)[1:]
    assert probe == scan and probe[3] == 0, (probe, scan)
    assert probe[1] == _oracle_count(oracle_for([W.UNIQUE_INGRESS_HOST], cs, extra), objs, nss) > 300
    b.free()
    d.put_data("/external/admission.k8s.gatekeeper.sh/namespace/ing-ns-00", [{"x": 1}])
    b = d.stage_objects(objs, nss)
    probe = cpu_baseline.sweep(d, b, threads=4)[1:]
    scan = cpu_baseline.sweep(d, b, threads=4, joins=False)[1:]
    assert probe == scan, (probe, scan)


def _ingresses_with_composite_hosts(n, seed):
    """gen_ingresses plus, on every fifth Ingress, a rule whose host is an
    object or array placed before the string hosts: the composite key value has
    no bucket and must not hide the string keys after it (devrt.h op_keyout)."""
    objs, nss = W.gen_ingresses(n, seed=seed)
    for i, o in enumerate(objs):
        if i % 5 == 0:
            o["spec"]["rules"].insert(0, {"host": {"x": i % 3}} if i % 2 else {"host": ["a", i % 4]})
    return objs, nss


def test_checker_composite_key_before_scalar_keys():
    """a leaf whose first key value is composite keeps its later string keys in
    the index: checker probe = scan = oracle, and nothing falls back"""
    from oracle import cpu_baseline
    objs, nss = _ingresses_with_composite_hosts(200, 12)
    cs = [W.constraint("K8sUniqueIngressHost", "uih")]
    extra = [(data_path(o), o) for o in objs]
    d = _driver([W.UNIQUE_INGRESS_HOST], cs, extra, host_only=True)
    b = d.stage_objects(objs, nss)
    probe = cpu_baseline.sweep(d, b, threads=4)[1:]
    scan = cpu_baseline.sweep(d, b, threads=4, joins=False)[1:]
    assert probe == scan and probe[3] == 0, (probe, scan)
    assert probe[1] == _oracle_count(oracle_for([W.UNIQUE_INGRESS_HOST], cs, extra), objs, nss) > 150


@pytest.mark.gpu
def test_composite_key_before_scalar_keys_on_gpu():
    """the same Ingresses on the device: rows equal the oracle's, the index is built"""
    objs, nss = _ingresses_with_composite_hosts(300, 13)
    cs = [W.constraint("K8sUniqueIngressHost", "uih")]
    extra = [(data_path(o), o) for o in objs]
    drv = gkgpu.Driver()
    rep, res = run_objects(drv, [W.UNIQUE_INGRESS_HOST], cs, objs, nss, extra_data=extra)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.fallback == 0 and rep.errors == 0 and rep.violations > 200, rep
    st = drv.join_stats()
    assert st["indexes"] == 1 and st["unindexed"] == 0, st


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [True, False])
def test_unique_ingress_host_join_on_gpu(jit):
    """the multi-valued join on the device (both back ends) equals the oracle;
    one index, entries for every distinct host of every Ingress"""
    objs, nss = W.gen_ingresses(400, seed=8)
    cs = [W.constraint("K8sUniqueIngressHost", "uih")]
    extra = [(data_path(o), o) for o in objs]
    drv = gkgpu.Driver(jit=jit)
    rep, res = run_objects(drv, [W.UNIQUE_INGRESS_HOST], cs, objs, nss, extra_data=extra)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.fallback == 0 and rep.errors == 0 and rep.violations > 300, rep
    st = drv.join_stats()
    assert st["indexes"] == 1 and st["unindexed"] == 0 and st["entries"] > len(objs), st


@pytest.mark.gpu
@pytest.mark.parametrize("jit", [True, False])
def test_join_index_matches_oracle_with_edge_keys(jit):
    """K8sJoinLabelParam over objects whose tag values are strings, numbers,
    booleans, null and objects (composite keys are in no bucket; numbers share
    one bucket): the probe path equals the oracle, on both device back ends."""
    vals = ["a", "b", 7, 7.0, True, None, {"x": 1}, "a", 3, False]
    objs = _labelled(120, 5, value=lambda r, i: vals[r.randint(0, len(vals) - 1)])
    cs = [W.constraint("K8sJoinLabelParam", "c", parameters={"label": "app"})]
    extra = [(data_path(o), o) for o in objs]
    drv = gkgpu.Driver(jit=jit)
    rep, res = run_objects(drv, [LABEL_PARAM], cs, objs, _ns(objs), extra_data=extra)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.fallback == 0 and rep.violations > 100, rep
    st = drv.join_stats()
    assert st["indexes"] == 1 and st["unindexed"] == 0 and st["entries"] > 0, st


@pytest.mark.gpu
def test_failing_key_pass_leaves_the_scan():
    """A synced Service whose selector holds a number: flatten_selector's
    concat fails on it in the key pass, so that constraint's site stays
    unindexed and its lanes scan -- reporting what the reference reports."""
    ts, cs = W.config2()
    ts = [t for t in ts if t["spec"]["crd"]["spec"]["names"]["kind"] == "K8sUniqueServiceSelector"]
    cs = [c for c in cs if c["kind"] == "K8sUniqueServiceSelector"]
    svcs = []
    for i in range(40):
        sel = {"app": "a%d" % (i % 6)}
        if i == 7:
            sel = {"app": 5}
        svcs.append({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "s%d" % i, "namespace": "ns-%d" % (i % 3)},
                     "spec": {"selector": sel}})
    extra = [(data_path(o), o) for o in svcs]
    drv = gkgpu.Driver()
    rep, res = run_objects(drv, ts, cs, svcs, _ns(svcs), extra_data=extra)
    assert not rep.mismatches, rep.mismatches[:3]
    st = drv.join_stats()
    assert st["indexes"] == 0 and st["unindexed"] == 1, st


@pytest.mark.gpu
def test_join_index_follows_inventory_changes():
    """puts and deletes of synced objects between evaluations: the indexes are
    rebuilt with the engine's state and the results stay the oracle's."""
    objs = _labelled(90, 9)
    cs = [W.constraint("K8sJoinLabelParam", "c", parameters={"label": "app"})]
    drv = _driver([LABEL_PARAM], cs)
    od = oracle_for([LABEL_PARAM], cs)
    reviews = [augmented_review(o, n) for o, n in zip(objs, _ns(objs))]
    entries = []
    for step in range(4):
        if step == 1:
            for o in objs[:50]:
                drv.put_data(data_path(o), o)
                od.put_data(data_path(o), json.dumps(o))
        if step == 2:
            for o in objs[:20]:
                drv.delete_data(data_path(o))
                od.delete_data(data_path(o))
        if step == 3:
            for o in objs:
                drv.put_data(data_path(o), o)
                od.put_data(data_path(o), json.dumps(o))
        rep = compare(od, reviews, drv.review_objects(objs, _ns(objs)))
        assert not rep.mismatches and rep.fallback == 0, (step, rep)
        entries.append(drv.join_stats()["entries"])
    assert entries[0] == 0 and entries[3] > entries[1] > entries[2] > 0, entries


@pytest.mark.gpu
def test_config6_probe_equals_scan_at_scale(monkeypatch):
    """config 6 at 3,000 objects (1,500 Services x 3,000 inventory leaves):
    every review's results with the join indexes equal the plain scan's
    (GKGPU_JOINS=0), emission order included."""
    objs_js, nss_js = W.gen_config6_json(3000)
    inv = W.inventory_paths(objs_js)
    objs = [json.loads(o) for o in objs_js]
    nss = [json.loads(n) for n in nss_js]
    ts, cs = W.config6()
    rows = {}
    for joins in ("1", "0"):
        monkeypatch.setenv("GKGPU_JOINS", joins)
        drv = _driver(ts, cs, [(p, json.loads(o)) for p, o in inv])
        res = drv.review_objects(objs, nss)
        assert not any(res.status[i] for i in range(len(objs)))
        rows[joins] = engine_rows(res, len(objs))
        if joins == "1":
            st = drv.join_stats()
            assert st["indexes"] == 3 and st["unindexed"] == 0 and st["entries"] > 3000, st
        else:
            assert drv.join_stats()["indexes"] == 0
    n = sum(len(r) for r in rows["1"])
    assert n > 1000
    for i in range(len(objs)):
        assert rows["1"][i] == rows["0"][i], (i, rows["1"][i][:3], rows["0"][i][:3])


def test_function_early_exit_keeps_results():
    """GKGPU_FN_EARLY=1 (compiler.cc early_exit_ok): a function whose bodies
    all yield one constant and cannot err stops at its first solution --
    probe_is_missing / missing / identical in the agilebank templates.  The
    CPU checker's result ROWS with it (an order-free digest of (review,
    constraint, message, details), oracle/cpuvm.cc gkcpu_sweep_digest) equal
    the oracle's on config 2 Pods and on config 6 (a subprocess: the switch is
    read once per process)."""
    import os
    import subprocess
    import sys
    code = r'''
import json, sys
sys.path[:0] = [%r, %r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, augmented_review
from oracle import cpu_baseline
from parity import oracle_for, oracle_review
def drv(ts, cs, extra=()):
    d = gkgpu.Driver(host_only=True); cl = Client(d)
    for t in ts: cl.add_template(t)
    for c in cs: cl.add_constraint(c)
    for p, o in extra: d.put_data(p, o)
    return d
def want_digest(d, od, objs, nss):
    cidx = {kn: i for i, kn in enumerate(d.constraints())}
    rows = []
    for i, (o, n) in enumerate(zip(objs, nss)):
        for kind, name, msg, det, _ea in oracle_review(od, augmented_review(o, n)):
            rows.append((i, cidx[(kind, name)], msg, det))
    return cpu_baseline.row_digest(rows), len(rows)
ts, cs = W.config2()
pods, ns_of, ns_objs = W.gen_pods(400, seed=9, n_namespaces=20)
nss = [ns_objs[n] for n in ns_of]
d = drv(ts, cs)
got = cpu_baseline.sweep_digest(d, d.stage_objects(pods, nss), threads=2)
want = want_digest(d, oracle_for(ts, cs), pods, nss)
ts6, cs6 = W.config6()
objs, onss = W.gen_config6_json(200)
inv = [(p, json.loads(o)) for p, o in W.inventory_paths(objs)]
d6 = drv(ts6, cs6, inv)
got6 = cpu_baseline.sweep_digest(d6, d6.stage_objects(objs, onss), threads=2)
want6 = want_digest(d6, oracle_for(ts6, cs6, inv), [json.loads(o) for o in objs], [json.loads(n) for n in onss])
print(json.dumps([got[1], got[2], got[3], want[0], want[1], got6[1], got6[2], got6[3], want6[0], want6[1]]))
''' % (os.path.join(ROOT, "gatekeeper-1_amd"), ROOT, os.path.join(ROOT, "tests"))
    for early in ("0", "1"):
        env = dict(os.environ, GKGPU_FN_EARLY=early)
        out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-2000:]
        v, fl, dg, wd, wn, v6, fl6, dg6, wd6, wn6 = json.loads(out.stdout.strip().splitlines()[-1])
        assert fl == 0 and fl6 == 0
        assert v == wn > 100 and v6 == wn6 > 20, (early, v, wn, v6, wn6)
        assert dg == wd and dg6 == wd6, (early, "row digests differ from the oracle's")
