"""Column form of staged batches (north_star "columnar, path-interned ...
arrays in HBM"; gatekeeper-1_amd/csrc/colplan.cc, colstore.cc).

The referenced-path plan of each compiled template decides what a staged
batch uploads: value columns for the paths the programs only navigate, node
subtrees for the paths they read whole.  The CPU checker (oracle/cpuvm.cc, the
device runtime built for the host) evaluates the column form exactly as the
device reads it (gk_debug_host_args_columns); its row digest must equal the
node form's and the oracle's (tests/parity.py rows), on the bench workloads
and on documents whose shapes break every assumption a schema could make
(paths that are arrays in one review and objects in the next, nulls, scalars
where objects are expected, duplicate keys, non-ASCII)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r'''
import json, sys, ctypes as C
sys.path[:0] = [%r, %r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, augmented_review
from gkgpu.page import Page
from oracle import cpu_baseline
from parity import oracle_for, oracle_review
cfg, n, edge = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3] == "1"
ts, cs = getattr(W, "config%%d" %% cfg)()
gen = {2: lambda: W.gen_pods_json(n, seed=42, n_namespaces=30, start=0),
       3: lambda: W.gen_config3_json(n, seed=7, start=0),
       4: lambda: W.gen_config4_json(n, seed=1234, start=0),
       6: lambda: W.gen_config6_json(n)}[cfg]
objs, nss = gen()
inv = W.inventory_paths(objs) if cfg == 6 else []
objs = [json.loads(o) for o in objs]
nss = [json.loads(x) if x else None for x in nss]
if edge:
    ns = {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": "edge", "labels": {"env": "dev"}}}
    odd = [
        {"spec": {"containers": {"a": {"name": "x", "image": "nginx"}}}},          # an object where an array is
        {"spec": {"containers": [None, 7, "s", [1, 2], {"name": None}]}},           # elements of every kind
        {"spec": {"containers": None, "initContainers": False}},
        {"spec": {"containers": [{"name": "c", "image": "openpolicyagent/opa:1",
                                  "resources": {"limits": {"cpu": 2, "memory": None}}}]}},
        {"spec": {"containers": [{"name": "c", "resources": {"limits": {"cpu": {"x": 1}, "memory": [1]}}}]}},
        {"spec": {"containers": [{"name": "c", "resources": []}, {"name": "d", "resources": "r"}]}},
        {"spec": {"containers": [{"name": "c", "readinessProbe": [], "livenessProbe": {"tcpSocket": False}}]}},
        {"spec": {"containers": [{"name": "c", "readinessProbe": None, "livenessProbe": {"exec": None}}]}},
        {"spec": {"containers": [{"name": "céK", "image": "gcr.io/x/opa:é", "readinessProbe": 3}]}},
        {"spec": []},
        {"spec": None, "metadata": {"labels": None}},
        {"metadata": {"labels": {"owner": 5, "app": None}}, "spec": {"containers": []}},
        {"metadata": {"labels": ["owner"]}, "spec": {"containers": [{}]}},
    ]
    for i, o in enumerate(odd):
        o = dict(o)
        md = dict(o.get("metadata") or {})
        md.update({"name": "edge-%%d" %% i, "namespace": "edge"})
        for kind in ("Pod", "Deployment", "Service", "ConfigMap"):
            objs.append(dict(o, apiVersion="v1", kind=kind, metadata=md))
            nss.append(ns)
    # duplicate keys: the flattener keeps document order, every reader takes the first
    dup = '{"apiVersion":"v1","kind":"Pod","metadata":{"name":"dup","namespace":"edge"},' \
          '"spec":{"containers":[{"name":"a","name":"b","image":"nginx","image":"openpolicyagent/x"}]}}'
d = gkgpu.Driver(host_only=True); cl = Client(d)
for t in ts: cl.add_template(t)
for c in cs: cl.add_constraint(c)
for path, js in inv: d.put_data(path, json.loads(js))
b = d.stage_page(Page.from_lists([json.dumps(o) for o in objs], [json.dumps(x) if x else None for x in nss]))
lib = d._lib
lib.gk_batch_columns.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.POINTER(C.c_uint64)]
why, nb = C.c_char_p(), C.c_uint64()
form = lib.gk_batch_columns(b._h, None, C.byref(why), C.byref(nb))
nodes = cpu_baseline.sweep_digest(d, b, threads=4)
cols = cpu_baseline.sweep_digest(d, b, threads=4, columns=True) if form == 1 else None
od = oracle_for(ts, cs, [(p, json.loads(js)) for p, js in inv]) if inv else oracle_for(ts, cs)
cidx = {kn: i for i, kn in enumerate(d.constraints())}
rows = []
for i, (o, ns) in enumerate(zip(objs, nss)):
    got = oracle_review(od, augmented_review(o, ns))
    if got == "ERROR":
        continue
    for kind, name, msg, det, _ea in got:
        rows.append((i, cidx[(kind, name)], msg, det))
print(json.dumps({"form": form, "why": (why.value or b"").decode(), "bytes": nb.value, "n": len(objs),
                  "nodes": list(nodes), "cols": list(cols) if cols else None,
                  "oracle": [cpu_baseline.row_digest(rows), len(rows)]}))
''' % (os.path.join(ROOT, "gatekeeper-1_amd"), ROOT, os.path.join(ROOT, "tests"))


def _run(cfg, n, edge):
    env = dict(os.environ, GKGPU_COLUMNS="1")
    out = subprocess.run([sys.executable, "-c", CODE, str(cfg), str(n), "1" if edge else "0"], env=env,
                         capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("cfg,n,edge", [(2, 600, False), (2, 300, True), (3, 600, False), (4, 500, False),
                                        (4, 300, True), (6, 400, False)])
def test_column_form_rows_equal_node_form_and_oracle(cfg, n, edge):
    r = _run(cfg, n, edge)
    assert r["form"] == 1, r["why"]
    ev, viol, flagged, dg = r["nodes"]
    assert r["cols"] == r["nodes"], ("column form differs from node form", r)
    # flagged pairs (CPU fallback) are the node form's own; the oracle
    # comparison holds for the configurations the bench runs without them
    if flagged == 0:
        assert [dg, viol] == r["oracle"], ("checker rows differ from the oracle's", r)
    assert viol > 50


def test_column_form_uploads_only_what_the_programs_read():
    """config 2's Pods: the referenced columns and the label objects the match
    stage scans, well under the node form's ~970 B per Pod"""
    r = _run(2, 2000, False)
    assert r["form"] == 1
    assert r["bytes"] / r["n"] < 400, r["bytes"] / r["n"]


PLAN_CODE = r'''
import sys, ctypes as C
sys.path[:0] = [%r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client
ts, cs = W.config2()
d = gkgpu.Driver(host_only=True); cl = Client(d)
for t in ts: cl.add_template(t)
lib = d._lib
lib.gk_debug_template_paths.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p)]
out = C.c_char_p()
assert lib.gk_debug_template_paths(d._e, b"K8sContainerLimits", C.byref(out)) == 0
print(out.value.decode())
''' % (os.path.join(ROOT, "gatekeeper-1_amd"), ROOT)


def test_container_limits_path_plan():
    """colplan.cc on k8scontainterlimits_template.yaml: `spec[field]` is a
    computed-key lookup, the containers are iterated, the limits object is
    looked up by computed key (missing(limits, "cpu")), the message prints
    only scalars -- so nothing above the leaves is read whole"""
    out = subprocess.run([sys.executable, "-c", PLAN_CODE], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    plan = out.stdout
    assert "review.object.spec [dyn]" in plan
    assert "review.object.spec[*] [iter]" in plan
    assert "review.object.spec[*][*].resources.limits [dyn]" in plan
    assert "NOT COLUMNAR" not in plan
    assert "review.object.spec[*][*] [" not in plan  # the container itself is never read whole
