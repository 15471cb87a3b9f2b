"""Minimal GPU probe: one tiny batch per workload, printed (used before the full suite)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from parity import run_objects  # noqa: E402

ts, cs = W.config1()
nss = W.gen_namespaces(8, seed=1)
rep, res = run_objects(gkgpu.Driver(), ts, cs, nss, [None] * len(nss))
print("config1", rep, [(r.review, r.msg, r.details_json) for r in res.results][:4], res.status, res.timing_ms)
ts, cs = W.config2()
pods, ns_of, ns_objs = W.gen_pods(16, seed=42, n_namespaces=4)
rep, res = run_objects(gkgpu.Driver(), ts, cs, pods, [ns_objs[n] for n in ns_of])
print("config2", rep, res.status, res.reason, res.timing_ms)
for m in rep.mismatches[:3]:
    print("MISMATCH", m)
