"""GPU probe: per-constraint fallback/error reasons on the config2 parity workload."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from parity import engine_for  # noqa: E402

ts, cs = W.config2()
pods, ns_of, ns_objs = W.gen_pods(1500, seed=42, n_namespaces=100)
nss = [ns_objs[n] for n in ns_of]
for i in range(len(cs)):
    d = gkgpu.Driver()
    engine_for(d, ts, [cs[i]])
    res = d.review_objects(pods, nss)
    cnt = collections.Counter((res.status[j], res.reason[j]) for j in range(len(pods)) if res.status[j])
    print(cs[i]["kind"], "violations", len(res.results), "flagged", dict(cnt))
