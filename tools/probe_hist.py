"""GPU probe: per-instruction execution histogram of one template (GKGPU_PROFILE=2)."""
import os
import sys

os.environ["GKGPU_PROFILE"] = "2"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
which = sys.argv[2] if len(sys.argv) > 2 else "K8sContainerLimits"
out = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/hist_%s.txt" % which
ts, cs = W.config2()
objs, nss = W.gen_pods_json(N, seed=42, n_namespaces=1000)
d = gkgpu.Driver()
cl = Client(d)
for t in ts:
    cl.add_template(t)
for c in cs:
    if c["kind"] == which:
        cl.add_constraint(c)
b = d.stage_objects(objs, nss)
r = b.eval(decode=False, light=True)
os.makedirs(os.path.dirname(out), exist_ok=True)
with open(out, "w") as f:
    f.write("# %d pods, %s, vm stats %s\n" % (N, which, r.vm_stats()))
    f.write(d.debug_disasm(which))
print("wrote", out, r.vm_stats())
