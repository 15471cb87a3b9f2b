"""GPU probe: per-step kernel times of repeated evaluations of one staged batch
(config 2), to check that bench.py's steady state matches a single launch."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
only = sys.argv[2] if len(sys.argv) > 2 else ""
ts, cs = W.config2()
if only:
    cs = [c for c in cs if c["kind"] == only]
objs, nss = W.gen_pods_json(N, seed=42, n_namespaces=1000)
d = gkgpu.Driver()
cl = Client(d)
for t in ts:
    cl.add_template(t)
for c in cs:
    cl.add_constraint(c)
b = d.stage_objects(objs, nss)
for i in range(12):
    t0 = time.perf_counter()
    r = b.eval(decode=False, light=True)
    wall = (time.perf_counter() - t0) * 1e3
    print("step %2d wall %.2f ms" % (i, wall), [(k, round(ms, 2)) for k, ms, n in r.launches], "tuples", r.device_tuples, "flagged", r.n_fallbacks + r.n_errors, flush=True)
import torch  # noqa: E402
_p = torch.cuda.get_device_properties(0)
print("sclk_mhz %.1f cus %d" % (d.debug_clock_mhz(), _p.multi_processor_count), flush=True)
