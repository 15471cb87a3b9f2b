"""The set-algebra rewrite of rule bodies (rego.cc optimize_sets,
GKGPU_REGO_SETS, a mask of two patterns): `v1 := {k | T[k]}; v2 := A - v1; count(v2) == count(A)` with
A a set rule becomes `not __gk_anyin(A, T)` -- k8srequiredprobes'
probe_field_empty (demo/agilebank/templates/k8srequiredprobes_template.yaml:36-40)
no longer builds two sets per container and probe.  The CPU checker's result
rows (oracle/cpuvm.cc gkcpu_sweep_digest) equal the oracle's with and without
the rewrite, on config 2 Pods and on probe values of every shape (missing,
scalar, empty object, false / non-false members, arrays with a numeric probe
type)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r'''
import copy, json, sys
sys.path[:0] = [%r, %r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, augmented_review
from oracle import cpu_baseline
from parity import oracle_for, oracle_review
ts, cs = W.config2()
ts = [t for t in ts if t["spec"]["crd"]["spec"]["names"]["kind"] == "K8sRequiredProbes"]
cs = [c for c in cs if c["kind"] == "K8sRequiredProbes"]
c2 = copy.deepcopy(cs[0])
c2["metadata"]["name"] = "odd-probe-types"
c2["spec"]["parameters"]["probeTypes"] = ["tcpSocket", 0, "exec"]
cs = cs + [c2]
pods, ns_of, ns_objs = W.gen_pods(300, seed=21, n_namespaces=10)
nss = [ns_objs[n] for n in ns_of]
shapes = [None, "x", {}, {"httpGet": False}, {"httpGet": {}}, {"exec": {"command": ["a"]}}, [True], [False, True],
          {"tcpSocket": None}, 7]
for i, s in enumerate(shapes):
    ctr = {"name": "c%%d" %% i, "image": "openpolicyagent/opa:0.9.2"}
    if s is not None:
        ctr["livenessProbe"] = s
        ctr["readinessProbe"] = s
    pods.append({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "shape-%%d" %% i, "namespace": "default"},
                 "spec": {"containers": [ctr]}})
    nss.append({"metadata": {"name": "default"}})
d = gkgpu.Driver(host_only=True); cl = Client(d)
for t in ts: cl.add_template(t)
for c in cs: cl.add_constraint(c)
got = cpu_baseline.sweep_digest(d, d.stage_objects(pods, nss), threads=2)
od = oracle_for(ts, cs)
cidx = {kn: i for i, kn in enumerate(d.constraints())}
rows = []
for i, (o, n) in enumerate(zip(pods, nss)):
    for kind, name, msg, det, _ea in oracle_review(od, augmented_review(o, n)):
        rows.append((i, cidx[(kind, name)], msg, det))
print(json.dumps([got[1], got[2], got[3], cpu_baseline.row_digest(rows), len(rows)]))
''' % (os.path.join(ROOT, "gatekeeper-1_amd"), ROOT, os.path.join(ROOT, "tests"))


def test_set_rewrite_keeps_required_probes_rows():
    for on in ("1", "2", "3", "0"):
        env = dict(os.environ, GKGPU_REGO_SETS=on)
        out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-2000:]
        v, fl, dg, wd, wn = json.loads(out.stdout.strip().splitlines()[-1])
        assert fl == 0 and v == wn > 100, (on, v, wn)
        assert dg == wd, (on, "row digests differ from the oracle's")


CODE_RL = r'''
import json, sys
sys.path[:0] = [%r, %r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, augmented_review
from oracle import cpu_baseline
from parity import oracle_for, oracle_review
ts, cs = W.config4()
keep = ("K8sRequiredLabels",)
ts = [t for t in ts if t["spec"]["crd"]["spec"]["names"]["kind"] in keep]
cs = [c for c in cs if c["kind"] in keep]
objs, nss = W.gen_config4_json(1500, seed=77)
objs = [json.loads(o) for o in objs]
nss = [json.loads(n) if n else None for n in nss]
# label shapes: none, empty, a false / null / numeric value, every key present
extra = [None, {}, {"owner": ""}, {"owner": "x", "app": "y", "team": "z", "env": "w"}]
for i, lb in enumerate(extra):
    md = {"name": "lbl-%%d" %% i, "namespace": "default"}
    if lb is not None:
        md["labels"] = lb
    objs.append({"apiVersion": "v1", "kind": "ConfigMap", "metadata": md})
    nss.append({"metadata": {"name": "default"}})
d = gkgpu.Driver(host_only=True); cl = Client(d)
for t in ts: cl.add_template(t)
for c in cs: cl.add_constraint(c)
got = cpu_baseline.sweep_digest(d, d.stage_objects(objs, nss), threads=2)
od = oracle_for(ts, cs)
cidx = {kn: i for i, kn in enumerate(d.constraints())}
rows = []
for i, (o, n) in enumerate(zip(objs, nss)):
    for kind, name, msg, det, _ea in oracle_review(od, augmented_review(o, n)):
        rows.append((i, cidx[(kind, name)], msg, det))
print(json.dumps([got[1], got[2], got[3], cpu_baseline.row_digest(rows), len(rows)]))
''' % (os.path.join(ROOT, "gatekeeper-1_amd"), ROOT, os.path.join(ROOT, "tests"))


def test_set_rewrite_keeps_required_labels_rows():
    """`missing := required - provided` with provided = {label | labels[label]}
    becomes a comprehension over `required` with a negated lookup; rows (with
    set-valued messages and details) equal the oracle's either way"""
    for on in ("1", "2", "3", "0"):
        env = dict(os.environ, GKGPU_REGO_SETS=on)
        out = subprocess.run([sys.executable, "-c", CODE_RL], env=env, capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-2000:]
        v, fl, dg, wd, wn = json.loads(out.stdout.strip().splitlines()[-1])
        assert fl == 0 and v == wn > 100, (on, v, wn)
        assert dg == wd, (on, "row digests differ from the oracle's")


# Bodies the rewrites must leave alone or keep exact: the comprehension's
# collection names a variable local to it (a wildcard, a named index), which
# the rewrite would hoist out of the comprehension; and the local-set form of
# the second pattern (A assigned a comprehension earlier in the body).
EDGE_REGO = """package k8sedgesets

want = {x | x := input.parameters.keys[_]}

violation[{"msg": msg}] {
  have := {k | input.review.object.spec.containers[_].env[k]}
  missing := want - have
  count(missing) > 0
  msg := sprintf("wildcard missing %v", [missing])
}

violation[{"msg": msg}] {
  got := {k | input.review.object.spec.containers[i].env[k]}
  miss := want - got
  count(miss) == count(want)
  msg := sprintf("named local: none of %v", [miss])
}

violation[{"msg": msg, "details": {"m": m2}}] {
  req := {l | l := input.parameters.keys[_]}
  prov := {k | input.review.object.metadata.labels[k]}
  m2 := req - prov
  count(m2) > 0
  msg := sprintf("local set missing %v", [m2])
}

violation[{"msg": msg}] {
  ann := {k | input.review.object.metadata.annotations[k]}
  d := want - ann
  count(d) == count(want)
  msg := "no wanted annotation"
}
"""

CODE_EDGE = r'''
import json, random, sys
sys.path[:0] = [%r, %r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, augmented_review
from oracle import cpu_baseline
from parity import oracle_for, oracle_review
ts = [W._tmpl("K8sEdgeSets", %r)]
cs = [W.constraint("K8sEdgeSets", "edge", match={"kinds": [{"apiGroups": [""], "kinds": ["Pod"]}]},
                   parameters={"keys": ["a", "b", "c"]})]
rng = random.Random(5)
vals = [True, False, None, 0, "", "x", {}, [1]]
objs, nss = [], []
for i in range(400):
    ctrs = []
    for j in range(rng.randint(0, 3)):
        c = {"name": "c%%d" %% j}
        if rng.random() < 0.8:
            c["env"] = {k: rng.choice(vals) for k in rng.sample("abcdz", rng.randint(0, 4))}
        ctrs.append(c)
    md = {"name": "p%%d" %% i, "namespace": "default"}
    if rng.random() < 0.8:
        # label values are strings (the match stage's labelSelector columns)
        md["labels"] = {k: rng.choice(["", "x"]) for k in rng.sample("abcz", rng.randint(0, 4))}
    if rng.random() < 0.7:
        md["annotations"] = {k: rng.choice(vals) for k in rng.sample("abcz", rng.randint(0, 3))}
    objs.append({"apiVersion": "v1", "kind": "Pod", "metadata": md, "spec": {"containers": ctrs}})
    nss.append({"metadata": {"name": "default"}})
d = gkgpu.Driver(host_only=True); cl = Client(d)
for t in ts: cl.add_template(t)
for c in cs: cl.add_constraint(c)
assert d.template_backend("K8sEdgeSets")[0] != 0, d.template_backend("K8sEdgeSets")
got = cpu_baseline.sweep_digest(d, d.stage_objects(objs, nss), threads=2)
od = oracle_for(ts, cs)
cidx = {kn: i for i, kn in enumerate(d.constraints())}
rows = []
for i, (o, n) in enumerate(zip(objs, nss)):
    for kind, name, msg, det, _ea in oracle_review(od, augmented_review(o, n)):
        rows.append((i, cidx[(kind, name)], msg, det))
print(json.dumps([got[1], got[2], got[3], cpu_baseline.row_digest(rows), len(rows)]))
''' % (os.path.join(ROOT, "gatekeeper-1_amd"), ROOT, os.path.join(ROOT, "tests"), EDGE_REGO)


def test_set_rewrite_refuses_comprehension_local_variables():
    """rego.cc closed_before: of the four bodies only the two whose
    collection is closed (metadata.labels, metadata.annotations) are
    rewritten; the rows equal the oracle's with the rewrites on and off."""
    for on in ("3", "0"):
        env = dict(os.environ, GKGPU_REGO_SETS=on, GKGPU_SETS_TRACE="1")
        out = subprocess.run([sys.executable, "-c", CODE_EDGE], env=env, capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-2000:]
        v, fl, dg, wd, wn = json.loads(out.stdout.strip().splitlines()[-1])
        assert fl == 0 and v == wn > 50, (on, v, wn)
        assert dg == wd, (on, "row digests differ from the oracle's")
        if on == "3":
            tr = [ln for ln in out.stderr.splitlines() if "optimize_sets" in ln and "K8sEdgeSets" in ln]
            assert tr and tr[0].endswith(": 2 rewrites"), out.stderr[-1500:]
