"""GPU probe: per-template fallback/error reasons on the config-5 webhook workload."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from parity import engine_for  # noqa: E402

ts, cs = W.config5(5)
ins = W.gen_admission_inputs(10)
for jit in (True, False):
    for i in range(len(cs)):
        d = gkgpu.Driver(jit=jit)
        engine_for(d, ts, [cs[i]])
        res = d.query_batch(ins)
        cnt = collections.Counter((res.status[j], res.reason[j]) for j in range(len(ins)) if res.status[j])
        print("jit" if jit else "vm", cs[i]["kind"], "violations", len(res.results), "flagged", dict(cnt), flush=True)
