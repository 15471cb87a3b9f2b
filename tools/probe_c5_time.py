"""GPU probe: where a config-5 webhook micro-batch (256 UPDATE AdmissionReviews
x 50 PSP constraints) spends its time: engine phases (flatten, upload, kernels,
download, decode) vs the Python wrapper, averaged over repeated calls."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ts, cs = W.config5(50)
d = gkgpu.Driver()
cl = Client(d)
for t in ts:
    cl.add_template(t)
for c in cs:
    cl.add_constraint(c)
bs = [W.gen_admission_inputs(batch, seed=99, start=i * batch) for i in range(8)]
for i in range(20):
    d.query_batch(bs[i % 8])
N = 200
ph = [0.0] * 5
wall = 0.0
nl = 0
kern = {}
for i in range(N):
    t0 = time.perf_counter()
    r = d.query_batch(bs[i % 8])
    wall += time.perf_counter() - t0
    for k in range(5):
        ph[k] += r.timing_ms[k]
    nl += len(r.launches)
    for k, ms, n in r.launches:
        kern[k] = kern.get(k, 0.0) + ms
print("wall %.3f ms/call; engine phases (flatten, upload, kernels, download, decode) ms:" % (wall / N * 1e3),
      [round(x / N, 3) for x in ph], "launches/call %.1f" % (nl / N))
for k, v in sorted(kern.items(), key=lambda kv: -kv[1]):
    print("  %-28s %.3f ms/call" % (k, v / N))
