"""Kernel resource usage of the template kernels (jit.cc) without a GPU.

Dumps the hipRTC source of every template kernel of a configuration
(GKGPU_JIT_DUMP_ONLY: the generator runs, hipRTC does not) and compiles each
with hipcc for gfx950 with -Rpass-analysis=kernel-resource-usage, which prints
the VGPR/SGPR counts, spills, the private-segment (scratch) bytes per lane,
LDS bytes and occupancy the code object will have on the device.

    python tools/jit_resources.py [--config 2] [--out profiles/r03_jit_resources.txt]
"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gatekeeper-1_amd", "csrc")


def dump_sources(config):
    d = tempfile.mkdtemp(prefix="gkjit_res")
    code = r'''
import sys
sys.path[:0] = [%r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client
ts, cs = getattr(W, "config%d")()
import os
for t in ts:
    # one engine per template: its kernel source alone in its own directory
    k = t["spec"]["crd"]["spec"]["names"]["kind"]
    os.makedirs(os.path.join(%r, k), exist_ok=True)
    os.environ["GKGPU_JIT_DUMP"] = os.path.join(%r, k)
    d = gkgpu.Driver()
    Client(d).add_template(t)
    print(k, d.template_backend(k))
''' % (ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), config, d, d)
    env = dict(os.environ, GKGPU_JIT_CACHE="0", GKGPU_JIT_DUMP=d, GKGPU_JIT_DUMP_ONLY="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    files = [(os.path.basename(os.path.dirname(f)), f) for f in sorted(glob.glob(os.path.join(d, "*", "*.hip")))]
    return files, r.stdout


FIELDS = ("VGPRs:", "AGPRs:", "SGPRs:", "ScratchSize", "Occupancy", "LDS Size", "VGPRs Spill", "SGPRs Spill")


def resources(path):
    src = open(path).read()
    name = re.search(r"__global__ void __launch_bounds__\([^)]*\) (gk_t_[0-9a-f]+)\(", src)
    out = path + ".o"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-w", "-mllvm", "-amdgpu-prealloc-sgpr-spill-vgprs", "--cuda-device-only",
                        "-c", "-I" + CSRC, "-Rpass-analysis=kernel-resource-usage", path, "-o", out],
                       capture_output=True, text=True, timeout=900)
    lines = [ln.split("remark: ")[-1] for ln in r.stderr.splitlines() if "remark:" in ln]
    keep = [ln for ln in lines if any(f in ln for f in FIELDS)]
    return (name.group(1) if name else os.path.basename(path)), r.returncode, keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    files, backends = dump_sources(a.config)
    rep = ["config %d template kernels (hipcc gfx950 -O3, kernel-resource-usage)" % a.config, backends.strip(), ""]
    for kind, f in files:
        name, rc, keep = resources(f)
        rep.append("%s %s (rc %d)" % (kind, name, rc))
        rep.extend("  " + k for k in keep)
    text = "\n".join(rep) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text)


if __name__ == "__main__":
    main()
