"""Offline check of the template kernels (no GPU): generate each workload
template's HIP source (GKGPU_JIT_DUMP), compile it with hipcc for gfx950 and
print the kernel resource usage (VGPRs, spills, scratch bytes per lane)."""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd")]

d = tempfile.mkdtemp(prefix="gkjit")
os.environ["GKGPU_JIT_CACHE"] = "0"
os.environ["GKGPU_JIT_DUMP"] = d
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "config2"
ts, cs = getattr(W, which)()
drv = gkgpu.Driver()
cl = Client(drv)
for t in ts:
    cl.add_template(t)
for c in cs:
    cl.add_constraint(c)
names = {}
for t in ts:
    k = t["spec"]["crd"]["spec"]["names"]["kind"]
    b, det = drv.template_backend(k)
    names[det] = k
    if b != 2:
        print(k, "NOT JIT:", det[:2000])
inc = os.path.join(ROOT, "gatekeeper-1_amd", "csrc")
for f in sorted(glob.glob(os.path.join(d, "*.hip"))):
    r = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-w", "-I", inc, "--cuda-device-only",
                        "-c", f, "-o", f + ".o", "-Rpass-analysis=kernel-resource-usage"],
                       capture_output=True, text=True)
    out = r.stderr
    m = re.search(r"Function Name: (\S+)", out)
    kn = m.group(1) if m else "?"
    vals = dict(re.findall(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|SGPRs Spill): (\d+)", out))
    print("%-22s %-24s rc=%d %s" % (names.get(kn, "?"), kn, r.returncode, vals))
    if r.returncode:
        print(out[-3000:])
