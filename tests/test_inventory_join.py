"""data.inventory joins on the engine's bytecode (CPU build of the device
runtime, oracle/cpuvm.cc) against the oracle, without a GPU.

demo/agilebank's unique-service-selector reads
`data.inventory.namespace[namespace][_]["Service"][name]`; the reference binds
data.inventory to data.external[target] (or {}) for every template evaluation
(vendor/.../frameworks/constraint/pkg/client/regolib/src.go:30-31,66-72).  The
engine assembles the synced objects into one tree in its permanent node
region (engine.cc sync_inventory).  The GPU parity tests compare per-review
results; here the host runtime's violation counts must equal the oracle's,
including after inventory puts and deletes."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd")]

import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client, augmented_review, data_path  # noqa: E402
from oracle import cpu_baseline  # noqa: E402
from parity import oracle_for, oracle_review  # noqa: E402


def _objects(n_svc, seed=3):
    import random
    rng = random.Random(seed)
    nss = ["ns-%d" % i for i in range(12)]
    ns_obj = {n: {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": n}} for n in nss}
    svcs, objs, objns = [], [], []
    for i in range(n_svc):
        ns = rng.choice(nss)
        sel = {"app": "app-%d" % rng.randint(0, 6)}
        if i % 5 == 0:
            sel["tier"] = rng.choice(["web", "db"])
        av = "v1" if i % 9 else "v2"
        s = {"apiVersion": av, "kind": "Service", "metadata": {"name": "svc-%d" % i, "namespace": ns},
             "spec": {"selector": sel}}
        svcs.append(s)
        objs.append(s)
        objns.append(ns_obj[ns])
    # a Service with no selector and one with an empty selector (flatten_selector -> "")
    for i, spec in enumerate(({}, {"selector": {}})):
        s = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "odd-%d" % i, "namespace": "ns-0"}, "spec": spec}
        svcs.append(s)
        objs.append(s)
        objns.append(ns_obj["ns-0"])
    return svcs, objs, objns


def _uss():
    ts, cs = W.config2()
    ts = [t for t in ts if t["spec"]["crd"]["spec"]["names"]["kind"] == "K8sUniqueServiceSelector"]
    cs = [c for c in cs if c["kind"] == "K8sUniqueServiceSelector"]
    return ts, cs


def _oracle_count(od, objs, objns):
    n = 0
    for o, ns in zip(objs, objns):
        r = oracle_review(od, augmented_review(o, ns))
        assert r != "ERROR"
        n += len(r)
    return n


def test_unique_service_selector_counts_match_oracle():
    ts, cs = _uss()
    svcs, objs, objns = _objects(120)
    extra = [(data_path(o), o) for o in svcs]
    d = gkgpu.Driver(host_only=True)
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    for p, o in extra:
        d.put_data(p, o)
    assert d.template_status("K8sUniqueServiceSelector")[0] == 1
    b = d.stage_objects(objs, objns)
    _, evals, viol, _, flagged = cpu_baseline.sweep(d, b, threads=2)
    want = _oracle_count(oracle_for(ts, cs, extra), objs, objns)
    assert flagged == 0
    assert want > 100
    assert viol == want


def test_inventory_tree_follows_puts_and_deletes():
    import json
    ts, cs = _uss()
    svcs, objs, objns = _objects(60, seed=5)
    d = gkgpu.Driver(host_only=True)
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    od = oracle_for(ts, cs)
    seen = []
    for step in range(4):
        if step == 1:
            for o in svcs[:30]:
                d.put_data(data_path(o), o)
                od.put_data(data_path(o), json.dumps(o))
        elif step == 2:
            for o in svcs[:10]:
                d.delete_data(data_path(o))
                od.delete_data(data_path(o))
        elif step == 3:
            for o in svcs:
                d.put_data(data_path(o), o)
                od.put_data(data_path(o), json.dumps(o))
        b = d.stage_objects(objs, objns)
        _, _, viol, _, flagged = cpu_baseline.sweep(d, b, threads=2)
        b.free()
        assert flagged == 0
        assert viol == _oracle_count(od, objs, objns), step
        seen.append(viol)
    assert seen[0] == 0 and seen[3] > seen[1] > 0


def _namespaces(n, seed=7):
    import random
    rng = random.Random(seed)
    out = []
    for i in range(n):
        labels = {}
        if rng.random() < 0.7:
            labels["gatekeeper"] = "v%d" % rng.randint(0, n // 3)
        out.append({"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "ns-%03d" % i, "labels": labels}})
    return out


def test_unique_label_counts_match_oracle():
    """demo/basic's K8sUniqueLabel (array.concat over both inventory scopes,
    `not identical_*` negations) on the host runtime vs the oracle, with the
    Namespaces synced as cluster-scoped inventory."""
    ts = [W.UNIQUE_LABEL]
    cs = [W.constraint("K8sUniqueLabel", "ns-gk-label-unique",
                       match={"kinds": [{"apiGroups": [""], "kinds": ["Namespace"]}]},
                       parameters={"label": "gatekeeper"})]
    # the template's inventory arrays and their concatenation are iterated
    # lazily (compiler.cc lazy arrays): no lane-heap limit on the inventory
    nss = _namespaces(150)
    extra = [(data_path(o), o) for o in nss]
    d = gkgpu.Driver(host_only=True)
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    for p, o in extra:
        d.put_data(p, o)
    assert d.template_status("K8sUniqueLabel")[0] == 1, d.template_status("K8sUniqueLabel")
    b = d.stage_objects(nss, [None] * len(nss))
    _, _, viol, _, flagged = cpu_baseline.sweep(d, b, threads=2)
    want = _oracle_count(oracle_for(ts, cs, extra), nss, [None] * len(nss))
    assert flagged == 0
    assert want >= 2
    assert viol == want


def test_config6_joins_without_lane_heap_fallback():
    """bench.py --config 6: agilebank's five constraints
    plus a unique-label constraint over synced Services and labelled
    Deployments that are also the reviewed objects.  unique-label's
    inventory arrays (cluster_objs / ns_objs / all_objs) are iterated lazily
    (compiler.cc lazy arrays), so no review falls back on the lane heap, and
    the host runtime's violation count equals the oracle's."""
    import json
    ts, cs = W.config6()
    objs, nss = W.gen_config6_json(160)
    inv = W.inventory_paths(objs)
    d = gkgpu.Driver(host_only=True)
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    for p, o in inv:
        d.put_data(p, o)
    b = d.stage_objects(objs, nss)
    _, evals, viol, _, flagged = cpu_baseline.sweep(d, b, threads=2)
    od = oracle_for(ts, cs, [(p, json.loads(o)) for p, o in inv])
    want = _oracle_count(od, [json.loads(o) for o in objs], [json.loads(n) for n in nss])
    assert flagged == 0
    assert evals == len(objs) * len(cs)
    assert viol == want and want > 50
