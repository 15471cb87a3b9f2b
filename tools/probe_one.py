"""GPU probe: one staged config2 sweep (all four templates), printed per launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ts, cs = W.config2()
objs, nss = W.gen_pods_json(N, seed=42, n_namespaces=1000)
d = gkgpu.Driver()
cl = Client(d)
for t in ts:
    cl.add_template(t)
for c in cs:
    cl.add_constraint(c)
kinds = {d.template_backend(t["spec"]["crd"]["spec"]["names"]["kind"])[1]: t["spec"]["crd"]["spec"]["names"]["kind"]
         for t in ts}
b = d.stage_objects(objs, nss)
for _ in range(reps):
    r = b.eval(decode=False, light=True)
    print([(kinds.get(ln.kernel, ln.kernel), round(ln.ms, 3), ln.tuples) for ln in r.launches], flush=True)
