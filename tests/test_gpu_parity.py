"""GPU parity: the HIP engine vs the CPU oracle on the same driver calls and inputs.

Bar: bit-exact (constraint, msg, details, enforcementAction) multisets per
review; the engine's CPU-fallback reviews are excluded and counted (they would
be evaluated by CPU OPA), and must stay a small fraction on these workloads.
"""
import json
import os

import pytest

import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, augmented_review, constraint_path

from parity import Report, compare, engine_for, oracle_for, oracle_review, run_objects

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module", autouse=True)
def _need_device():
    if not gkgpu.Driver.device_available():
        pytest.fail("no HIP device visible: GPU parity tests must run on an MI355X")


_BACKEND = {"jit": True}


@pytest.fixture(autouse=True, params=["jit", "vm"])
def backend(request):
    """every parity test runs on both device back ends: the per-template
    hipRTC kernels (jit.cc) and the bytecode VM kernel (kernels.hip)"""
    _BACKEND["jit"] = request.param == "jit"
    yield request.param


def Driver():
    d = gkgpu.Driver(jit=_BACKEND["jit"])
    return d


def _assert_backend(drv, kinds, guard=()):
    want = 2 if _BACKEND["jit"] else 1
    for k in kinds:
        b, detail = drv.template_backend(k)
        assert b == (3 if k in guard else want), (k, b, detail)


def _assert_clean(rep, max_fallback_frac=0.0):
    assert not rep.mismatches, rep.mismatches[:3]
    # byte-exact: no test using _assert_clean reviews object-printing templates
    assert rep.canonical_only == 0, rep
    assert rep.compared > 0
    total = rep.compared + rep.fallback + rep.errors
    assert rep.fallback <= max_fallback_frac * total, rep


def test_config1_namespaces_required_labels():
    ts, cs = W.config1()
    nss = W.gen_namespaces(10000, seed=1)  # BASELINE configs[0]: all 10k Namespaces
    rep, res = run_objects(Driver(), ts, cs, nss, [None] * len(nss))
    _assert_clean(rep)
    assert rep.violations > 1000
    # README.md:313-327 message shape
    assert any(r.msg == 'you must provide labels: {"gatekeeper"}' for r in res.results)
    assert all(r.details_json == '{"missing_labels":["gatekeeper"]}' for r in res.results)


def test_config2_agilebank_pods():
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(1500, seed=42, n_namespaces=100)
    nss = [ns_objs[n] for n in ns_of]
    drv = Driver()
    rep, res = run_objects(drv, ts, cs, pods, nss)
    _assert_clean(rep)
    assert rep.violations > 5000
    _assert_backend(drv, [t["spec"]["crd"]["spec"]["names"]["kind"] for t in ts])
    kernels = {k for k, _, _ in res.launches}
    # deferred messages sized and formatted by the size / format passes (kernels.hip)
    # (tuples from per-wave slot chunks packed first: gk_compact)
    passes = {"gk_compact", "gk_size_kernel", "gk_scan_spine", "gk_format_kernel"}
    assert passes <= kernels, res.launches
    kernels -= passes
    if _BACKEND["jit"]:
        assert kernels and all(k.startswith("gk_t_") for k in kernels), res.launches
    else:
        assert kernels == {"audit_kernel"}, res.launches


def _pods_services_deployments(seed=44, n_pods=1500, n_svc=300, n_dep=100):
    import random
    pods, ns_of, ns_objs = W.gen_pods(n_pods, seed=seed, n_namespaces=60)
    objs = list(pods)
    nss = [ns_objs[n] for n in ns_of]
    rng = random.Random(3)
    names = sorted(ns_objs)
    svcs = []
    for i in range(n_svc):
        ns = rng.choice(names)
        av = "v1" if i % 10 else "v2"
        sel = {"app": "app-%d" % rng.randint(0, 9)}
        if i % 7 == 0:
            sel["tier"] = rng.choice(["web", "db"])
        svcs.append({"apiVersion": av, "kind": "Service", "metadata": {"name": "svc-%d" % i, "namespace": ns},
                     "spec": {"selector": sel}})
        nss.append(ns_objs[ns])
    objs += svcs
    for i in range(n_dep):
        ns = rng.choice(names)
        objs.append({"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d-%d" % i, "namespace": ns}})
        nss.append(ns_objs[ns])
    return pods, svcs, objs, nss


def test_config2_unique_service_selector_join_on_gpu():
    """All five demo/agilebank constraints over Pods + Services + Deployments,
    with the Services synced into the inventory (target.go ProcessData paths).
    unique-service-selector's data.inventory join (regolib src.go:30-31,66-72)
    and sort run on the device: no review falls back, and every review's
    results equal the oracle's (manager.go:376-380 per object)."""
    from gkgpu.client import data_path
    ts, cs = W.config2()
    assert len(cs) == 5
    pods, svcs, objs, nss = _pods_services_deployments()
    extra = [(data_path(o), o) for o in svcs]
    drv = Driver()
    rep, res = run_objects(drv, ts, cs, objs, nss, extra_data=extra)
    import collections
    reasons = collections.Counter(res.reason[i] for i in range(len(objs)) if res.status[i])
    if _BACKEND["jit"]:
        assert rep.fallback == 0, (rep, reasons)
        _assert_clean(rep)
    else:
        # the bytecode VM formats each message into the lane's 4 KB buffer at
        # emission (no deferred records): Services sharing a selector with
        # dozens of others exceed it and go to the CPU fallback (FB_MSG_LEN)
        assert set(reasons) <= {2}, reasons
        assert not rep.mismatches, rep.mismatches[:3]
        assert rep.fallback <= 0.05 * len(objs), rep
    per = {}
    for v in res.results:
        per[v.constraint_name] = per.get(v.constraint_name, 0) + 1
    assert per.get("unique-service-selector", 0) > 500, per
    assert rep.violations > 5000
    _assert_backend(drv, [t["spec"]["crd"]["spec"]["names"]["kind"] for t in ts])


@pytest.mark.parametrize("compact", [False, True])
def test_unique_service_selector_inventory_changes(monkeypatch, compact):
    """The inventory tree follows put/delete of synced objects between sweeps.
    compact: GKGPU_COMPACT_MIN=0 compacts the permanent node region (constraints,
    namespaces, template constants and the inventory tree re-placed, templates
    recompiled) whenever its garbage exceeds its live nodes -- here at every
    rebuild -- and the results stay the oracle's."""
    from gkgpu.client import data_path
    if compact:
        monkeypatch.setenv("GKGPU_COMPACT_MIN", "0")
    ts, cs = W.config2()
    _, svcs, objs, nss = _pods_services_deployments(seed=45, n_pods=50, n_svc=80, n_dep=5)
    drv = Driver()
    engine_for(drv, ts, cs)
    od = oracle_for(ts, cs)
    reviews = [augmented_review(o, n) for o, n in zip(objs, nss)]
    sizes = []
    for step in range(5):
        if step == 1:
            for o in svcs[:40]:
                drv.put_data(data_path(o), o)
                od.put_data(data_path(o), json.dumps(o))
        if step == 2:
            for o in svcs[:20]:
                drv.delete_data(data_path(o))
                od.delete_data(data_path(o))
        if step >= 3:
            for o in svcs[20 + step:40 + step]:
                drv.put_data(data_path(o), o)
                od.put_data(data_path(o), json.dumps(o))
            for c in cs:  # re-put: the old constraint documents become garbage
                drv.put_data(constraint_path(c), c)
        rep = compare(od, reviews, drv.review_objects(objs, nss))
        _assert_clean(rep)
        sizes.append(drv.debug_store_sizes()[0])
    if compact:
        assert sizes[-1] <= 2 * sizes[0] + 50000, sizes


def test_unique_label_join_on_gpu(monkeypatch):
    """demo/basic's K8sUniqueLabel (data.inventory over both scopes,
    array.concat, negated helper calls) over Namespaces synced as inventory:
    results equal the oracle's.  Its inventory arrays are iterated lazily
    (compiler.cc lazy arrays), so no lane falls back at any inventory size;
    with the lazy path switched off (GKGPU_LAZY_ARRAYS=0) the lane heap holds
    them and beyond a few dozen objects the lanes go to the CPU fallback
    (FB_HEAP) -- still bit-exact for the rest."""
    import random
    from gkgpu.client import data_path
    ts = [W.UNIQUE_LABEL]
    cs = [W.constraint("K8sUniqueLabel", "ns-gk-label-unique",
                       match={"kinds": [{"apiGroups": [""], "kinds": ["Namespace"]}]},
                       parameters={"label": "gatekeeper"})]
    for n, lazy, want_fb in ((12, "1", False), (60, "1", False), (400, "1", False), (60, "0", True)):
        monkeypatch.setenv("GKGPU_LAZY_ARRAYS", lazy)
        rng = random.Random(n)
        nss = []
        for i in range(n):
            labels = {"gatekeeper": "v%d" % rng.randint(0, n // 3)} if rng.random() < 0.7 else {}
            nss.append({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "ns-%03d" % i, "labels": labels}})
        drv = Driver()
        rep, res = run_objects(drv, ts, cs, nss, [None] * n, extra_data=[(data_path(o), o) for o in nss])
        assert not rep.mismatches, rep.mismatches[:3]
        if want_fb:
            assert rep.fallback > 0 and all(res.reason[i] == 1 for i in range(n) if res.status[i] & 2), rep
        else:
            assert rep.fallback == 0 and rep.violations >= 2, rep
        _assert_backend(drv, ["K8sUniqueLabel"])


GUARDED = W._tmpl("K8sGuardedEncode", """package k8sguardedencode

violation[{"msg": msg}] {
	input.review.kind.kind == "Service"
	input.review.kind.version == "v1"
	input.review.kind.group == ""
	x := base64.encode(input.review.object.metadata.name)
	msg := sprintf("encoded <%v>", [x])
}
""")


def test_guard_program_routes_only_matching_reviews_to_cpu():
    """A template outside the subset (base64.encode) runs as a guard program:
    its kind/version/group tests run on the device after the match, so only
    v1 Services are flagged for CPU fallback; Pods, apps/v1 Deployments and v2
    Services are evaluated on the GPU, bit-exact with the oracle."""
    ts, cs = W.config2()
    ts = ts + [GUARDED]
    cs = cs + [{"apiVersion": "constraints.gatekeeper.sh/v1beta1", "kind": "K8sGuardedEncode",
                "metadata": {"name": "guarded"}}]
    pods, svcs, objs, nss = _pods_services_deployments()
    n_svc = sum(1 for s in svcs if s["apiVersion"] == "v1")
    drv = Driver()
    rep, res = run_objects(drv, ts, cs, objs, nss)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.fallback == n_svc, rep
    assert all(res.status[i] == 0 for i in range(len(pods)))
    assert all(res.reason[i] == 12 for i in range(len(objs)) if res.status[i] & 2)  # FB_TEMPLATE
    assert rep.violations > 5000
    _assert_backend(drv, [t["spec"]["crd"]["spec"]["names"]["kind"] for t in ts], guard=("K8sGuardedEncode",))


def test_config2_output_buffers_grow(monkeypatch):
    """Output capacities far below the call's output (GKGPU_TEST_CAPS: tuples,
    staged bytes, output bytes of a new evaluation context): the tuple /
    staged-byte overflow re-runs the evaluation with grown buffers, the output
    byte overflow re-runs only the size + format passes; results are unchanged."""
    monkeypatch.setenv("GKGPU_TEST_CAPS", "64,256,1024")
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(600, seed=43, n_namespaces=50)
    nss = [ns_objs[n] for n in ns_of]
    rep, res = run_objects(Driver(), ts, cs, pods, nss)
    _assert_clean(rep)
    assert rep.violations > 1000
    assert res.device_tuples > 64 and res.device_bytes > 1024


def test_config2_agilebank_namespaces_regex():
    ts, cs = W.config2()
    nss = W.gen_namespaces(2000, seed=7)
    rep, res = run_objects(Driver(), ts, cs, nss, [None] * len(nss))
    _assert_clean(rep)
    msgs = {r.msg for r in res.results}
    assert "All namespaces must have an `owner` label that points to your company username" in msgs


def test_demo_agilebank_resources():
    """Shapes of demo/agilebank/{bad,good}_resources."""
    ts, cs = W.config2()
    pods = [
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "opa", "namespace": "production"},
         "spec": {"containers": [{"name": "opa", "image": "openpolicyagent/opa:0.9.2",
                                  "args": ["run", "--server", "--addr=localhost:8080"],
                                  "resources": {"limits": {"cpu": "300m", "memory": "4000Mi"}}}]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "opa", "namespace": "production"},
         "spec": {"containers": [{"name": "opa", "image": "openpolicyagent/opa:0.9.2"}]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "opa", "namespace": "production"},
         "spec": {"containers": [{"name": "opa", "image": "gcr.io/smythe-kpc/testbuilds/opa:0.9.2",
                                  "resources": {"limits": {"cpu": "100m", "memory": "30Mi"}}}]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "opa", "namespace": "production"},
         "spec": {"containers": [{"name": "opa", "image": "openpolicyagent/opa:0.9.2",
                                  "resources": {"limits": {"cpu": "100m", "memory": "30Mi"}},
                                  "readinessProbe": {"httpGet": {"path": "/", "port": 8080}},
                                  "livenessProbe": {"tcpSocket": {"port": 8080}}}]}},
        W.namespace_obj("production", {"owner": "me"}),
        W.namespace_obj("production", {"owner": "me.agilebank.demo"}),
    ]
    nss = [W.namespace_obj("production")] * 4 + [None, None]
    rep, res = run_objects(Driver(), ts, cs, pods, nss)
    _assert_clean(rep)
    per = [[r.msg for r in res.results if r.review == i] for i in range(len(pods))]
    assert "container <opa> cpu limit <300m> is higher than the maximum allowed of <200m>" in per[0]
    assert per[1].count("container <opa> has no resource limits") == 2  # two rules, no dedupe
    assert any("invalid image repo" in m for m in per[2])
    assert per[3] == []
    assert per[5] == []


def _integration_reviews(case):
    o = case["object"]
    obj = {"apiVersion": "%s/v1" % o["group"], "kind": o["kind"]}
    if o.get("labels"):
        obj["metadata"] = {"labels": o["labels"]}
    ns = case["namespace"]
    nsobj = None
    if ns is not None:
        md = {"name": ns["name"], "creationTimestamp": None}
        if ns.get("labels"):
            md["labels"] = ns["labels"]
        nsobj = {"metadata": md, "spec": {}, "status": {}}
    kind = {"group": o["group"], "version": "v1", "kind": o["kind"]}
    base = {"uid": "", "kind": kind, "resource": {"group": "", "version": "", "resource": ""}}
    if ns is not None:
        base["namespace"] = ns["name"]
    tail = {"operation": "", "userInfo": {}}
    unstable = {"namespace": nsobj} if nsobj is not None else {}
    r1 = dict(base, **tail, object=obj, oldObject=None, options=None, _unstable=unstable)
    r2 = dict(base, **tail, object=None, oldObject=obj, options=None, _unstable=unstable)
    r3 = dict(base, **tail, object=obj, oldObject=None, options=None, _unstable=unstable)
    return [r1, r2, r3]


def test_target_integration_cases():
    """pkg/target/target_integration_test.go:141-363, three review forms each."""
    cases = json.load(open(os.path.join(HERE, "golden", "integration_cases.json")))
    deny_all = W._tmpl("DenyAll", 'package denyall\n\nviolation[{"msg": msg}] {\n\tmsg := "denyall constraint installed"\n}\n')
    rep = Report()
    for case in cases:
        c = W.constraint("DenyAll", "my-constraint", match=case["match"])
        drv = Driver()
        cl = Client(drv)
        cl.add_template(deny_all)
        cl.add_constraint(c)
        od = oracle_for([deny_all], [c])
        reviews = _integration_reviews(case)
        res = drv.query_batch([{"review": r} for r in reviews])
        compare(od, reviews, res, rep)
        for i in range(3):
            got_allowed = not any(r.review == i for r in res.results)
            assert res.status[i] == 0, case["name"]
            assert got_allowed == case["allowed"], (case["name"], i)
    assert not rep.mismatches, rep.mismatches[:3]


def test_label_and_annotation_regex_config3():
    ts = [W.ALLOWED_LABEL_REGEX, W.ALLOWED_ANNOTATION_REGEX]
    rules = [{"key": "env", "allowedRegex": "^(dev|stage|prod)-[0-9]{1,4}$"},
             {"key": "owner", "allowedRegex": "^[a-zA-Z]+.agilebank.demo$"},
             {"key": "app", "allowedRegex": "^[a-z0-9]([-a-z0-9]*[a-z0-9])?$"}]
    cs = [W.constraint("K8sAllowedLabelRegex", "label-rules",
                       match={"kinds": [{"apiGroups": ["apps", ""], "kinds": ["Deployment", "Service"]}]},
                       parameters={"rules": rules}),
          W.constraint("K8sAllowedAnnotationRegex", "annotation-rules",
                       match={"kinds": [{"apiGroups": ["apps", ""], "kinds": ["Deployment", "Service"]}]},
                       parameters={"rules": rules})]
    import random
    rng = random.Random(7)
    vals = {"env": ["dev-1", "prod-9999", "prod-10000", "stage-", "dev-12\n", "qa-1", ""],
            "owner": ["alice.agilebank.demo", "bob_agilebank.demo", "x.agilebank.demo\n", "9.agilebank.demo"],
            "app": ["web", "-web", "web-", "a", "Web", "a-b-c", ""]}
    objs = []
    for i in range(1500):
        kind = rng.choice(["Deployment", "Service"])
        lab = {k: rng.choice(v) for k, v in vals.items() if rng.random() < 0.8}
        ann = {k: rng.choice(v) for k, v in vals.items() if rng.random() < 0.5}
        objs.append({"apiVersion": "apps/v1" if kind == "Deployment" else "v1", "kind": kind,
                     "metadata": {"name": "o%d" % i, "namespace": "ns%d" % (i % 7), "labels": lab, "annotations": ann}})
    nss = [W.namespace_obj("ns%d" % (i % 7)) for i in range(len(objs))]
    rep, res = run_objects(Driver(), ts, cs, objs, nss)
    _assert_clean(rep)
    assert rep.violations > 500


def test_query_single_review_and_batch_agree():
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(50, seed=3, n_namespaces=5)
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    reviews = [augmented_review(p, ns_objs[n]) for p, n in zip(pods, ns_of)]
    batch = drv.query_batch([{"review": r} for r in reviews])
    objs = drv.review_objects(pods, [ns_objs[n] for n in ns_of])
    for i, r in enumerate(reviews):
        single = cl.review(r)
        a = sorted((x.constraint_name, x.msg) for x in single.results)
        b = sorted((x.constraint_name, x.msg) for x in batch.results if x.review == i)
        c = sorted((x.constraint_name, x.msg) for x in objs.results if x.review == i)
        assert a == b == c


def test_staged_batch_matches_direct_and_counts():
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(400, seed=5, n_namespaces=30)
    nss = [ns_objs[n] for n in ns_of]
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    direct = drv.review_objects(pods, nss)
    b = drv.stage_objects(pods, nss)
    r1 = b.eval(decode=True)
    r2 = b.eval(decode=False)
    assert sorted((x.review, x.msg) for x in r1.results) == sorted((x.review, x.msg) for x in direct.results)
    assert r2.totals == r1.totals
    assert sum(r1.totals) == len(r1.results)


def test_staged_batch_through_the_pinned_bounce_upload(monkeypatch):
    """The node arena of a staged batch goes to HBM through the pinned bounce
    buffers (engine.cc upload_bounce; by default only copies >= 256 MB, i.e.
    the bench's 1M Pods): with the threshold lowered, a multi-chunk upload of a
    smaller batch gives the same results as the direct path."""
    monkeypatch.setenv("GKGPU_BOUNCE_MIN", str(1 << 16))
    monkeypatch.setenv("GKGPU_BOUNCE_CHUNK", str(1 << 18))  # ~14 chunks, both buffers reused
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(3000, seed=8, n_namespaces=40)
    nss = [ns_objs[n] for n in ns_of]
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    direct = drv.review_objects(pods, nss)
    b = drv.stage_objects(pods, nss)
    r1 = b.eval(decode=True)
    assert len(r1.results) > 5000
    assert sorted((x.review, x.constraint_name, x.msg) for x in r1.results) == \
        sorted((x.review, x.constraint_name, x.msg) for x in direct.results)


def test_staged_batches_are_independent():
    """A staged batch keeps its own device documents: staging another batch or
    serving a Query in between does not change its results."""
    ts, cs = W.config2()
    pods_a, ns_a, nso_a = W.gen_pods(300, seed=11, n_namespaces=20)
    pods_b, ns_b, nso_b = W.gen_pods(200, seed=12, n_namespaces=20)
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    nss_a = [nso_a[n] for n in ns_a]
    nss_b = [nso_b[n] for n in ns_b]
    want_a = sorted((x.review, x.constraint, x.msg) for x in drv.review_objects(pods_a, nss_a).results)
    want_b = sorted((x.review, x.constraint, x.msg) for x in drv.review_objects(pods_b, nss_b).results)
    ba = drv.stage_objects(pods_a, nss_a)
    bb = drv.stage_objects(pods_b, nss_b)
    drv.review_objects(pods_b[:7], nss_b[:7])
    got_a = sorted((x.review, x.constraint, x.msg) for x in ba.eval(decode=True).results)
    got_b = sorted((x.review, x.constraint, x.msg) for x in bb.eval(decode=True).results)
    assert got_a == want_a
    assert got_b == want_b


def test_audit_writer_engine_matches_oracle():
    """status.violations / totalViolations / per-action totals written from the
    engine's results equal those written from the oracle's (manager.go:462-631)."""
    from gkgpu.audit import AuditWriter, resource_of
    from parity import engine_for, oracle_review
    ts, cs = W.config2()
    cs = [dict(c) for c in cs]
    cs[3] = W.constraint("K8sRequiredProbes", "must-have-probes", match=cs[3]["spec"]["match"],
                         parameters=cs[3]["spec"]["parameters"], enforcement_action="dryrun")
    pods, ns_of, ns_objs = W.gen_pods(600, seed=21, n_namespaces=30)
    nss = [ns_objs[n] for n in ns_of]
    drv = Driver()
    engine_for(drv, ts, cs)
    od = oracle_for(ts, cs)
    res = drv.review_objects(pods, nss)
    assert not any(res.status)
    resources = [resource_of(p) for p in pods]
    cons = drv.constraints()
    we = AuditWriter(cons)
    we.add_results(res.results, resources)
    wo = AuditWriter(cons)
    cidx = {kc: i for i, kc in enumerate(cons)}
    for i, p in enumerate(pods):
        for kind, name, msg, _det, ea in oracle_review(od, augmented_review(p, nss[i])):
            wo.add(cidx[(kind, name)], resources[i], msg, ea)
    assert we.statuses() == wo.statuses()
    assert we.per_action == wo.per_action
    assert we.per_action["dryrun"] > 0 and we.per_action["deny"] > 0


def test_device_output_copy_decodes_to_results():
    """Batch.eval(device_out=...) hands the raw gk_viol records + message bytes
    to caller device buffers (the tensors the multi-GPU gather sends)."""
    import torch
    from gkgpu.parallel import DeviceOutput, decode
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(300, seed=31, n_namespaces=20)
    nss = [ns_objs[n] for n in ns_of]
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    b = drv.stage_objects(pods, nss)
    out = DeviceOutput(torch.device("cuda", 0))
    r = b.eval(decode=False, light=True, device_out=out)
    assert out.n_tuples == r.device_tuples and out.n_bytes == r.device_bytes
    rows = decode([(out.tuples(), out.bytes())])
    full = b.eval(decode=True)
    assert [(x[0], x[1], x[4]) for x in rows] == [(x.review, x.constraint, x.msg) for x in full.results]


def test_device_output_drops_rows_of_flagged_reviews():
    """the raw device output handed to a gather holds only the rows
    of reviews the engine answered -- not those of reviews that fall back to
    CPU OPA (non-ASCII subjects under a `.` pattern, config 3) nor those of a
    constraint whose enforcementAction is not a string (the Query errors) -- so
    the gathered rows equal the decode path's rows."""
    import torch
    from gkgpu.parallel import DeviceOutput, decode
    from parity import engine_for
    ts, cs = W.config3()
    cs = [json.loads(json.dumps(c)) for c in cs]
    cs[3]["spec"]["enforcementAction"] = 7  # invalid: Query returns an error for reviews it matches
    objs, nss = W.gen_config3_json(300, seed=5)
    objs = [json.loads(o) for o in objs]
    nss = [json.loads(n) for n in nss]
    extra = [{"apiVersion": "v1", "kind": "Service",
              "metadata": {"name": "u%d" % i, "namespace": "c3-ns-000", "labels": {"owner": v, "env": "dev-1"},
                           "annotations": {"app": v}}}
             for i, v in enumerate(["émile.agilebank.demo", "日本", "xé"])]
    objs += extra
    nss += [nss[0]] * len(extra)
    drv = Driver()
    engine_for(drv, ts, cs)
    b = drv.stage_objects(objs, nss)
    full = b.eval(decode=True)
    assert any(st & 2 for st in full.status) and any(st & 1 for st in full.status)
    out = DeviceOutput(torch.device("cuda", 0))
    r = b.eval(decode=False, light=True, device_out=out)
    assert out.n_tuples < r.device_tuples
    rows = decode([(out.tuples(), out.bytes())])
    assert [(x[0], x[1], x[4]) for x in rows] == [(x.review, x.constraint, x.msg) for x in full.results]


@pytest.mark.parametrize("order", ["0", "1", None])
def test_config4_staged_batch_every_match_order(monkeypatch, order):
    """staged batches reorder reviews (kind first, match-affinity
    signature, size; GKGPU_MATCH_ORDER 0 = size only, 1 = signature first,
    default 2).  Config 4's mixed kinds x 50 randomized constraints through
    stage + eval under each order, against the oracle, and the raw device
    output decoded (parallel.decode) equal to the decoded results."""
    import torch
    from gkgpu.parallel import DeviceOutput, decode
    from parity import engine_for
    if order is None:
        monkeypatch.delenv("GKGPU_MATCH_ORDER", raising=False)
    else:
        monkeypatch.setenv("GKGPU_MATCH_ORDER", order)
    ts, cs = W.config4()
    objs, nss = W.gen_config4_json(400, seed=4321)
    objs = [json.loads(o) for o in objs]
    nss = [None if n is None else json.loads(n) for n in nss]
    drv = Driver()
    engine_for(drv, ts, cs)
    od = oracle_for(ts, cs)
    b = drv.stage_objects(objs, nss)
    res = b.eval(decode=True)
    rep = compare(od, [augmented_review(o, n) for o, n in zip(objs, nss)], res)
    _assert_clean(rep)
    assert rep.violations > 500
    out = DeviceOutput(torch.device("cuda", 0))
    b.eval(decode=False, light=True, device_out=out)
    rows = decode([(out.tuples(), out.bytes())])
    assert [(x[0], x[1], x[4]) for x in rows] == [(x.review, x.constraint, x.msg) for x in res.results]


def test_config3_generator_regex_constraints():
    """Config 3's 10 allowedRegex constraints over its generator's Deployments
    and Services, plus non-ASCII subjects: those under a UTF-8-sensitive
    pattern (`.`) are routed to the CPU fallback, every other review is
    bit-exact with the oracle."""
    ts, cs = W.config3()
    objs, nss = W.gen_config3_json(700, seed=7)
    objs = [json.loads(o) for o in objs]
    nss = [json.loads(n) for n in nss]
    extra = [{"apiVersion": "v1", "kind": "Service",
              "metadata": {"name": "u%d" % i, "namespace": "c3-ns-000", "labels": {"owner": v, "env": "dev-1"},
                           "annotations": {"app": v}}}
             for i, v in enumerate(["émile.agilebank.demo", "bob.agilebank.demo", "日本", "xé"])]
    objs += extra
    nss += [nss[0]] * len(extra)
    rep, res = run_objects(Driver(), ts, cs, objs, nss)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.violations > 1000
    assert rep.fallback <= len(extra)


def test_config4_mixed_kinds_fifty_constraints():
    """Config 4: mixed kinds (Pods, Deployments, Services, ConfigMaps,
    Namespaces) x 50 constraints with randomized match blocks (namespaces,
    excludedNamespaces, label/namespace selectors, scope) and parameters."""
    ts, cs = W.config4()
    objs, nss = W.gen_config4_json(400, seed=1234)
    objs = [json.loads(o) for o in objs]
    nss = [None if n is None else json.loads(n) for n in nss]
    drv = Driver()
    rep, res = run_objects(drv, ts, cs, objs, nss)
    _assert_clean(rep)
    assert rep.violations > 500
    _assert_backend(drv, [t["spec"]["crd"]["spec"]["names"]["kind"] for t in ts])


def test_config5_webhook_micro_batch():
    """Config 5: 256 UPDATE AdmissionReviews (object + oldObject) per
    gk_query_batch launch over the PSP policies at constraint load 50."""
    from gkgpu.webhook import DENIED, handle_batch
    ts, cs = W.config5(50)
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    _assert_backend(drv, [t["spec"]["crd"]["spec"]["names"]["kind"] for t in ts])
    od = oracle_for(ts, cs)
    ins = W.gen_admission_inputs(256, seed=99)
    res = drv.query_batch(ins)
    rep = compare(od, [json.loads(s)["review"] for s in ins], res)
    _assert_clean(rep)
    assert rep.violations >= 256 * 10
    resp = handle_batch(drv, ins)
    assert all(r.code == DENIED for r in resp)
    # the bulk export (gk_results_export) carries exactly the per-row views
    from gkgpu.driver import export_rows
    blob, st = drv.query_batch_export(ins)
    rows = export_rows(blob)
    assert [(r[0], r[2], r[3]) for r in rows] == [(x.review, x.msg, x.details_json) for x in res.results]
    assert list(st) == list(res.status)


def test_format_pass_lds_windows_keep_bytes(monkeypatch):
    """The format pass stages each wavefront's output bytes in LDS windows
    (kernels.hip gk_format_kernel); with a 256-B window every wave's range
    spans many windows and tuples straddle window edges.  Rows equal the
    default window's and the oracle's (config 5: ~160-B PSP messages)."""
    ts, cs = W.config5(20)
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    ins = W.gen_admission_inputs(128, seed=7)
    base = drv.query_batch(ins)
    monkeypatch.setenv("GKGPU_FMT_STAGE", "256")
    small = drv.query_batch(ins)
    monkeypatch.delenv("GKGPU_FMT_STAGE")
    assert len(base.results) > 128
    assert [(x.review, x.msg, x.details_json) for x in small.results] == \
        [(x.review, x.msg, x.details_json) for x in base.results]
    rep = compare(oracle_for(ts, cs), [json.loads(s)["review"] for s in ins], small)
    _assert_clean(rep)


STR_BUILTINS = W._tmpl("K8sStrBuiltins", """package k8sstrbuiltins

violation[{"msg": msg}] {
	v := input.review.object.metadata.labels[k]
	parts := split(v, input.parameters.sep)
	t := trim(v, "-._")
	msg := sprintf("%v|%v|%v|%v|%v|%v|%v|%v|%v", [k, parts, t, lower(v), upper(k), concat("+", parts), indexof(v, "a"), trim_suffix(trim_prefix(v, "x"), "z"), count(parts)])
}
""")


def test_string_builtins_trim_split_case_concat_indexof():
    """trim / split / lower / upper / concat / indexof / trim_prefix /
    trim_suffix (topdown/strings.go) on adversarial label values; non-ASCII
    subjects of lower/upper and empty-separator splits go to the CPU."""
    import random
    rng = random.Random(11)
    vals = ["", "-", "--a--", "a.b.c", "xAbz", "x", "z", "xz", "a..b.", ".a.", "AbC-d_e", "...", "Héllo", "é",
            "ab.ab.ab", "-_.x._-", "aaaa"]
    objs = []
    for i in range(300):
        labels = {"k%d" % j: rng.choice(vals) for j in range(rng.randint(0, 4))}
        if rng.random() < 0.3:
            labels["Mixed-Key"] = rng.choice(vals)
        objs.append({"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm-%d" % i, "namespace": "ns",
                                                                         "labels": labels}})
    ns = W.namespace_obj("ns")
    cs = [W.constraint("K8sStrBuiltins", "dot", parameters={"sep": "."}),
          W.constraint("K8sStrBuiltins", "empty-sep", parameters={"sep": ""}),
          W.constraint("K8sStrBuiltins", "ab", parameters={"sep": "ab"})]
    drv = Driver()
    rep, _ = run_objects(drv, [STR_BUILTINS], cs, objs, [ns] * len(objs))
    _assert_backend(drv, ["K8sStrBuiltins"])
    _assert_clean(rep, max_fallback_frac=0.6)
    assert rep.violations > 500


def test_emission_argument_list_read_elsewhere():
    """ADVICE r05 (jit.cc dce_sites): a sprintf argument list that is also
    added into another array the body reads must be built (the emission-only
    list DCE must not fire); rows equal the oracle's on both back ends"""
    from test_jit_source import ALIASED_LIST, PLAIN_LIST
    ts = [W._tmpl("K8sAliasedList", ALIASED_LIST), W._tmpl("K8sPlainList", PLAIN_LIST)]
    cs = [W.constraint("K8sAliasedList", "aliased"), W.constraint("K8sPlainList", "plain")]
    objs = [{"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "cm-%d" % i, "namespace": "ns"}}
            for i in range(200)]
    drv = Driver()
    rep, res = run_objects(drv, ts, cs, objs, [W.namespace_obj("ns")] * len(objs))
    _assert_backend(drv, ["K8sAliasedList", "K8sPlainList"])
    _assert_clean(rep)
    assert rep.violations == 400, rep


def test_go_regex_whitespace_and_case_folding_on_device():
    """re_match as Go decides it (topdown/regex.go:21-34): `\\s` excludes \\v,
    and (?i) folds k / s with U+212A / U+017F -- decided by the device's DFA
    tables (no fallback: neither pattern is utf8-sensitive)"""
    ts = [W.ALLOWED_LABEL_REGEX]
    rules = [{"key": "note", "allowedRegex": "^[a-z]+(\\s[a-z0-9]+)*$"},
             {"key": "kube", "allowedRegex": "(?i)^(kube|sys)-[a-z]+$"}]
    cs = [W.constraint("K8sAllowedLabelRegex", "go-rules", match={"kinds": [{"apiGroups": [""], "kinds": ["Service"]}]},
                       parameters={"rules": rules})]
    notes = ["ok go", "ok\tgo", "ok\vgo", "ok\ngo", "ok go\v", "x\x0cy", "ok\u00a0go"]
    kubes = ["kube-ops", "KUBE-ops", "\u212aube-ops", "\u017fys-x", "kube-\u212a\u017f", "ube-x", "\u0130kube-x",
             "sys-\u00e9"]
    objs = []
    for i in range(len(notes) * len(kubes)):
        lab = {"note": notes[i % len(notes)], "kube": kubes[i // len(notes)]}
        objs.append({"apiVersion": "v1", "kind": "Service", "metadata": {"name": "s%d" % i, "namespace": "ns",
                                                                        "labels": lab}})
    drv = Driver()
    rep, res = run_objects(drv, ts, cs, objs, [W.namespace_obj("ns")] * len(objs))
    _assert_clean(rep)
    assert rep.fallback == 0, rep
    bad = {r.msg.split(">")[0] for r in res.results}
    assert "label <note: ok\vgo" in bad and "label <note: ok go" not in bad
    assert "label <kube: \u212aube-ops" not in bad and "label <kube: \u0130kube-x" in bad


def test_template_kernel_matches_vm_at_scale():
    """Size-independent property at 100k Pods (config 2 policies): the template
    kernels + format pass over size-ordered reviews produce exactly the
    violation multiset of the bytecode VM with in-kernel formatting in batch
    order, and repeat evaluations are identical."""
    if not _BACKEND["jit"]:
        pytest.skip("compares the two back ends; runs once")
    import collections
    import os
    ts, cs = W.config2()
    objs, nss = W.gen_pods_json(100_000, seed=42, n_namespaces=1000)

    def sweep(jit, fpass):
        old = os.environ.get("GKGPU_FORMAT_PASS")
        old_so = os.environ.get("GKGPU_SIZE_ORDER")
        os.environ["GKGPU_FORMAT_PASS"] = "1" if fpass else "0"
        os.environ["GKGPU_SIZE_ORDER"] = "1" if fpass else "0"
        try:
            d = gkgpu.Driver(jit=jit)
            cl = Client(d)
            for t in ts:
                cl.add_template(t)
            for c in cs:
                cl.add_constraint(c)
            b = d.stage_objects(objs, nss)
            out = [collections.Counter((x.review, x.constraint_name, x.msg, x.details_json) for x in b.eval().results)
                   for _ in range(2)]
            b.free()
            return out
        finally:
            for k, v in (("GKGPU_FORMAT_PASS", old), ("GKGPU_SIZE_ORDER", old_so)):
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    import sys
    import time
    t0 = time.time()
    vm = sweep(False, False)
    print("scale test: VM sweeps %.1f s" % (time.time() - t0), file=sys.stderr, flush=True)
    t0 = time.time()
    jit = sweep(True, True)
    print("scale test: JIT sweeps %.1f s" % (time.time() - t0), file=sys.stderr, flush=True)
    assert vm[0] == vm[1]
    assert sum(vm[0].values()) > 250_000
    assert jit[0] == jit[1]
    assert jit[0] == vm[0]


def _audit_rows_oracle(od):
    from oracle.driver import details_json
    rows = []
    for r in od.query('hooks["%s"].audit' % gkgpu.client.TARGET):
        rv, c = r["review"], r["constraint"]
        ns = rv.get("namespace") if hasattr(rv, "get") else None
        rows.append((rv.get("kind").get("kind"), ns if isinstance(ns, str) else "", rv.get("name"), c.get("kind"),
                     c.get("metadata").get("name"), r["msg"], details_json(r["details"]), r["enforcementAction"]))
    return rows


def test_audit_from_cache_inventory():
    """Client.Audit (client.go:805-833) -> hooks.audit over the synced inventory
    (target_template_source.go:46-89 make_review / add_field): reviews carry no
    _unstable.namespace, so namespace matching reads the synced Namespace cache.
    The engine enumerates the inventory in path order; rows are compared as a
    multiset (the reference iterates Go maps)."""
    from gkgpu.client import data_path
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(300, seed=5, n_namespaces=12)
    objs = list(ns_objs.values()) + pods
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    od = oracle_for(ts, cs)
    paths = []
    for o in objs:
        cl.add_data(o)
        od.put_data(data_path(o), json.dumps(o))
        paths.append(data_path(o))
    res = cl.audit()
    assert not any(res.status), "audit reviews flagged for fallback/error"
    order = sorted(set(paths))
    eng = []
    for r in res.results:
        seg = order[r.review].split("/")
        ns = seg[4] if seg[3] == "namespace" else ""
        eng.append((seg[-2], ns, seg[-1], r.constraint_kind, r.constraint_name, r.msg, r.details_json,
                    r.enforcement_action))
    ref = _audit_rows_oracle(od)
    assert len(ref) > 0
    assert sorted(eng) == sorted(ref)
    # removing an object drops exactly its rows (DeleteData on the inventory path)
    gone = pods[0]
    cl.remove_data(gone)
    od.delete_data(data_path(gone))
    res2 = cl.audit()
    n_gone = sum(1 for row in ref if row[2] == gone["metadata"]["name"] and row[1] == gone["metadata"]["namespace"])
    assert len(res2.results) == len(ref) - n_gone


def test_empty_and_degenerate_inputs():
    """Edges the reference handles without error: empty batches, an empty
    inventory, a null Query input, no constraints, and objects with missing or
    mistyped metadata (local.go:302-359; target.go:129-163)."""
    ts, cs = W.config2()
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    # no constraints yet: every path returns nothing
    assert drv.review_objects([W.namespace_obj("a")], [None]).results == []
    for c in cs:
        cl.add_constraint(c)
    assert drv.review_objects([], []).results == []
    assert drv.query_batch([]).results == []
    assert cl.audit().results == []
    b = drv.stage_objects([], [])
    assert b.eval().results == []
    b.free()
    # null input: hooks.violation binds no review -> no results, no error
    assert drv.query('hooks["%s"].violation' % gkgpu.client.TARGET, None).results == []
    odd = [
        {"apiVersion": "v1", "kind": "Pod"},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": 7, "namespace": ["x"]}, "spec": None},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "production"},
         "spec": {"containers": []}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "q", "namespace": "production"},
         "spec": {"containers": [{}]}},
        {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "r", "namespace": "production"},
         "spec": {"containers": [{"name": "c", "image": "", "resources": {"limits": {}}}]}},
        {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "n", "labels": {}}},
        {},
    ]
    nss = [None, None, W.namespace_obj("production"), W.namespace_obj("production"),
           W.namespace_obj("production"), None, None]
    rep, _ = run_objects(Driver(), ts, cs, odd, nss)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.compared + rep.fallback + rep.errors == len(odd)


def test_review_page_and_staged_page_match_objects_path():
    """The bulk List-page entry points (gk_review_page / gk_batch_stage_page,
    parallel host flattening) give the char** path's results, bit for bit."""
    from gkgpu.page import Page
    ts, cs = W.config2()
    objs, nss = W.gen_pods_json(5000, seed=9, n_namespaces=40)
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    key = lambda res: sorted((x.review, x.constraint, x.msg, x.details_json) for x in res.results)  # noqa: E731
    want = key(drv.review_objects(objs, nss))
    pg = Page.from_lists(objs, nss)
    assert key(drv.review_page(pg)) == want
    b = drv.stage_page(pg)
    assert key(b.eval(decode=True)) == want
    assert b.timing_ms()[1] > 0
    b.free()


def test_excluder_skips_audit_namespaces():
    """Excluder.IsNamespaceExcluded(Audit, ns) (excluder.go:82-86) in the
    audit loop (manager.go:362-365): objects of an excluded namespace are not
    reviewed (status GK_REVIEW_EXCLUDED, no results); the rest are unchanged."""
    from gkgpu.driver import GK_REVIEW_EXCLUDED
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(800, seed=17, n_namespaces=30)
    nss = [ns_objs[n] for n in ns_of]
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    full = drv.review_objects(pods, nss)
    drv.excluder_add(["audit"], ["production"])
    part = drv.review_objects(pods, nss)
    b = drv.stage_objects(pods, nss)
    staged = b.eval(decode=True)
    drv.excluder_add(["webhook"], ["team-0003"])  # invalidates the staged batch
    with pytest.raises(RuntimeError, match="state changed"):
        b.eval(decode=True)
    ex = {i for i, n in enumerate(ns_of) if n == "production"}
    assert ex and len(ex) < len(pods)
    for res in (part, staged):
        assert {i for i, s in enumerate(res.status) if s & GK_REVIEW_EXCLUDED} == ex
        got = sorted((x.review, x.constraint, x.msg) for x in res.results)
        assert got == sorted((x.review, x.constraint, x.msg) for x in full.results if x.review not in ex)
    assert b.excluded() == len(ex)


def test_batch_resource_is_handle_violation_identity():
    """gk_batch_resource == HandleViolation's Resource (target.go:193-244) for
    the staged reviews: apiVersion from review.kind, object metadata name/ns."""
    from gkgpu.target import handle_violation, resource_identity
    objs, nss = W.gen_config4_json(600, seed=77)
    objs = [json.loads(o) for o in objs]
    nss = [None if n is None else json.loads(n) for n in nss]
    objs.append({"apiVersion": "a/b/c", "kind": "Weird", "metadata": {"name": 5}})
    nss.append(None)
    ts, cs = W.config4()
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    b = drv.stage_objects(objs, nss)
    for i in list(range(0, len(objs), 37)) + [len(objs) - 1]:
        want = resource_identity(handle_violation(augmented_review(objs[i], nss[i])))
        assert b.resource(i) == want, i
    b.free()


def test_client_review_sets_handle_violation_resource():
    ts, cs = W.config2()
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    pods, ns_of, ns_objs = W.gen_pods(20, seed=3, n_namespaces=3)
    rv = augmented_review(pods[0], ns_objs[ns_of[0]])
    res = cl.review(rv)
    assert res.results
    for r in res.results:
        assert r.resource["apiVersion"] == "v1" and r.resource["kind"] == "Pod"
        assert r.resource["metadata"]["name"] == pods[0]["metadata"]["name"]


def test_match_kats_replayed_through_the_device():
    """Every function-level vector of the reference's match-library KATs
    (pkg/target/regolib/*_test.rego via tests/golden/match_kats.jsonl) as a
    (constraint, review, namespace cache) triple under a deny-all template,
    evaluated on the MI355X (gk_batch_eval of a staged batch of Query inputs
    and gk_query_batch): the rows equal the oracle's, including the
    autoreject branch (devrt.h audit_body, target_template_source.go:12-25)
    and match errors; for `direct` vectors the deny-all row appears iff the
    KAT's own result is true."""
    from kat_replay import UNDEF, cases, engine_for, expected, query_input
    cs = cases()
    n_auto = n_direct = 0
    for case in cs:
        want = expected(case)
        drv = Driver()
        engine_for(drv, case)
        for res in (drv.query_batch([query_input(case)]), drv.debug_stage_inputs([query_input(case)]).eval()):
            if want == "ERROR":
                assert res.status[0] & 1, case["id"]
                continue
            assert res.status[0] == 0, case["id"]
            got = sorted((r.msg, r.details_json, r.enforcement_action) for r in res.results)
            assert got == want, (case["id"], got, want)
        if want != "ERROR" and case["fn"] == "autoreject_review":
            n_auto += sum(1 for w in want if w[0] == "Namespace is not cached in OPA.")
        if want != "ERROR" and case["fn"] != "autoreject_review" and isinstance(case["kat"], bool):
            denied = any(w[0] == "denied" for w in want)
            if case["fn"] == "matches_label_selector" or denied == case["kat"]:
                n_direct += 1
                assert denied == case["kat"], case["id"]
    assert n_auto >= 1
    assert n_direct >= 60  # 61 function-level vectors with a boolean result


def _reverse_keys(v):
    """the same document with every object's members in reverse order (one
    of the Go map iteration orders OPA may see, ast/term.go:79-92)"""
    if isinstance(v, dict):
        return {k: _reverse_keys(v[k]) for k in reversed(list(v))}
    if isinstance(v, list):
        return [_reverse_keys(x) for x in v]
    return v


def test_psp_object_printing_messages_compare_canonically():
    """PSP messages %v-print objects (input.parameters, securityContext,
    volume).  The oracle gets every review and constraint with object members
    in reverse order -- a legal Go-map order of the reference -- while the
    engine keeps document order: the rows must agree after canonicalising the
    printed objects (tests/canonical.py), and some must differ byte-wise."""
    from canonical import canonical_row
    ts, cs = W.config5(20)
    drv = Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    od = oracle_for(ts, [_reverse_keys(c) for c in cs])
    ins = W.gen_admission_inputs(256, seed=7)
    reviews = [json.loads(s)["review"] for s in ins]
    res = drv.query_batch(ins)
    rep = compare(od, [_reverse_keys(r) for r in reviews], res)
    assert not rep.mismatches, rep.mismatches[:2]
    assert rep.canonical_only > 0, rep
    assert rep.violations > 256


def test_template_with_libs_bats_container_limits():
    """A template whose helpers are a lib (the reference's bats
    K8sContainerLimits, tests/golden/bats_fixtures.json): libs rewritten under
    libs.<target>.<Kind> as regorewriter does (client.go:280-347), compiled
    into the template kernel, bit-exact with the oracle over 1500 Pods plus the
    bats Pods, whose outcomes are test.bats:130-134's (no limits denied)."""
    bats = json.load(open(os.path.join(HERE, "golden", "bats_fixtures.json")))
    pods, ns_of, ns_objs = W.gen_pods(1500, seed=88, n_namespaces=20)
    objs = [p["object"] for p in bats["pods"]] + pods
    nss = [{"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": p["namespace"]}} for p in bats["pods"]]
    nss += [ns_objs[n] for n in ns_of]
    drv = Driver()
    rep, res = run_objects(drv, [bats["template"]], [bats["constraint"]], objs, nss)
    _assert_clean(rep)
    assert rep.violations > 1000
    _assert_backend(drv, ["K8sContainerLimits"])
    denied = {r.review for r in res.results}
    for i, p in enumerate(bats["pods"]):
        assert (i in denied) == p["denied"]


@pytest.mark.parametrize("fuse", ["1", "0"])
def test_emission_order_is_topdown_order(monkeypatch, fuse):
    """Within a (review, constraint) the engine's rows come in the order topdown
    emits them: body by body of the partial set, each body in iteration order.
    K8sContainerLimits' eight general_violation bodies share their first
    expression, so the compiler fuses them into one pass over the containers
    (GKGPU_FUSE, compiler.cc rule_group) and the OP_ORD keys restore the order
    (devrt.h op_ord / flush_wave)."""
    monkeypatch.setenv("GKGPU_FUSE", fuse)
    ts, cs = W.config2()
    t = [x for x in ts if x["spec"]["crd"]["spec"]["names"]["kind"] == "K8sContainerLimits"]
    c = [x for x in cs if x["kind"] == "K8sContainerLimits"]
    _check_emission_order(t, c, fuse)
    # the bats template: eight top-level violation bodies (fused in run())
    bats = json.load(open(os.path.join(HERE, "golden", "bats_fixtures.json")))
    _check_emission_order([bats["template"]], [bats["constraint"]], fuse)


def _check_emission_order(t, c, fuse):
    pods, ns_of, ns_objs = W.gen_pods(800, seed=515, n_namespaces=10)
    pods.append({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p", "namespace": "default"},
                 "spec": {"containers": [{"name": "a", "image": "x"},
                                         {"name": "b", "resources": {"limits": {"cpu": "9", "memory": "9Gi"}}},
                                         {"name": "c", "resources": {"limits": {"cpu": "zz"}}}]}})
    nss = [ns_objs[n] for n in ns_of] + [{"metadata": {"name": "default"}}]
    drv = Driver()
    rep, res = run_objects(drv, t, c, pods, nss)
    _assert_clean(rep)
    prog = drv.debug_disasm("K8sContainerLimits")
    assert (" ORD " in prog) == (fuse == "1")
    od = oracle_for(t, c)
    got = [[] for _ in pods]
    for r in res.results:
        got[r.review].append(r.msg)
    multi = 0
    for i, (p, n) in enumerate(zip(pods, nss)):
        want = [row[2] for row in oracle_review(od, augmented_review(p, n))]
        assert got[i] == want, (i, got[i], want)
        multi += len(want) > 1
    assert multi > 100


@pytest.mark.gpu
def test_config6_joins_on_gpu_equal_the_oracle():
    """bench.py --config 6 at 400 objects: agilebank's five constraints plus
    demo/basic unique-label over synced Services and labelled Deployments that
    are also the reviewed objects; every review's results equal the oracle's
    and no review falls back (lazy inventory arrays, memoized per-object join
    keys on the device)."""
    ts, cs = W.config6()
    objs_js, nss_js = W.gen_config6_json(300)
    objs = [json.loads(o) for o in objs_js]
    nss = [json.loads(n) for n in nss_js]
    extra = [(p, json.loads(o)) for p, o in W.inventory_paths(objs_js)]
    drv = Driver()
    rep, res = run_objects(drv, ts, cs, objs, nss, extra_data=extra)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.fallback == 0 and rep.errors == 0, rep
    assert rep.violations > 60, rep


def _heavy_pods(n, seed=3, cap=400):
    """Pods whose container count is heavy-tailed (Pareto, alpha 0.9, capped):
    most have one or two containers, a few dozen have hundreds"""
    import random
    rng = random.Random(seed)
    pool = [W._container(rng, "c%d" % i) for i in range(512)]
    objs, nss = [], []
    for i in range(n):
        k = min(cap, int(rng.paretovariate(0.9)))
        conts = []
        for j in range(k):
            c = dict(pool[rng.randrange(len(pool))])
            c["name"] = "c%d" % j
            conts.append(c)
        objs.append({"apiVersion": "v1", "kind": "Pod",
                     "metadata": {"name": "p%d" % i, "namespace": "team-1", "labels": {"app": "a"}},
                     "spec": {"containers": conts}})
        nss.append(W.namespace_obj("team-1", {"env": "dev"}))
    return objs, nss


def test_heavy_tailed_pods_fall_back_only_past_the_lane_limits():
    """the lane limits (heap words, byte buffer, 256
    emissions per lane) send a review to the CPU fallback.  On a heavy-tailed
    Pod distribution (1-400 containers) every review the engine keeps equals
    the oracle's, and only Pods with many containers fall back (reported)."""
    ts, cs = W.config2()
    objs, nss = _heavy_pods(1200)
    drv = Driver()
    rep, res = run_objects(drv, ts, cs, objs, nss)
    assert not rep.mismatches, rep.mismatches[:3]
    sizes = [len(o["spec"]["containers"]) for o in objs]
    fb = [sizes[i] for i in range(len(objs)) if res.status[i] & 2]
    floor = 64 if _BACKEND["jit"] else 8
    print("heavy-tailed pods: %d of %d fall back (container counts %s); %d > 100 containers" %
          (len(fb), len(objs), sorted(fb)[:12], sum(1 for s in sizes if s > 100)))
    assert all(s >= floor for s in fb), sorted(fb)
    assert rep.compared >= len(objs) - len(fb) - rep.errors
