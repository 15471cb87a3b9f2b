"""Kernel resource usage of the template kernels (jit.cc) without a GPU.

Compiles every template kernel of a configuration with hipRTC, exactly as the
engine does (jit.cc kOpts, gfx950), into a scratch code-object cache, and
reads each code object's metadata notes (llvm-readelf --notes): VGPRs, AGPRs,
SGPRs, their spill counts, the private-segment (scratch) bytes per lane, LDS
bytes per block, and the waves per SIMD the VGPR count allows.

    python tools/jit_resources.py [--config 2] [--out profiles/r05/r05_jit_resources_c2.txt]
"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
FIELDS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
          ".private_segment_fixed_size", ".group_segment_fixed_size", ".uses_dynamic_stack")


def compile_kernels(config, cache):
    code = r'''
import sys
sys.path[:0] = [%r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client
ts, cs = getattr(W, "config%d")()
d = gkgpu.Driver(host_only=True)
cl = Client(d)
for t in ts:
    cl.add_template(t)
for t in ts:
    k = t["spec"]["crd"]["spec"]["names"]["kind"]
    print(k, *d.template_backend(k))
''' % (ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), config)
    env = dict(os.environ, GKGPU_JIT_CACHE=cache)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=1800)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    out = {}
    for ln in r.stdout.splitlines():
        p = ln.split()
        if len(p) == 3:
            out[p[2]] = (p[0], p[1])
    return out


def notes(path):
    """per kernel entry of amdhsa.kernels (an entry starts at its `  - .` line:
    .agpr_count and .group_segment_fixed_size come before .name)"""
    r = subprocess.run([READELF, "--notes", path], capture_output=True, text=True)
    kernels, cur, name = {}, {}, None

    def close():
        if name and name.startswith("gk_t_"):
            kernels[name] = dict(cur)

    for ln in r.stdout.splitlines():
        if re.match(r"^  - \.", ln):  # a new kernel entry (argument entries are indented deeper)
            close()
            cur, name = {}, None
        m = re.search(r"^\s+\.name:\s+(\S+)", ln)
        if m:
            name = m.group(1)
        for f in FIELDS:
            m = re.search(re.escape(f) + r":\s+(\S+)", ln)
            if m:
                cur[f[1:]] = m.group(1)
    close()
    return kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    cache = tempfile.mkdtemp(prefix="gkjit_res")
    names = compile_kernels(a.config, cache)
    found = {}
    for co in glob.glob(os.path.join(cache, "*.co")):
        found.update(notes(co))
    rep = ["config %d template kernels: hipRTC code objects (jit.cc kOpts, gfx950), metadata notes" % a.config, ""]
    for name, (kind, backend) in names.items():
        k = found.get(name)
        rep.append("%s %s (backend %s)" % (kind, name, backend))
        if not k:
            rep.append("  no code object (bytecode VM)")
            continue
        # .vgpr_count is the unified total on gfx950 (arch VGPRs aligned to 4,
        # then the AGPRs: .agpr_count of them); 512 per SIMD lane, granule 8
        regs = int(k.get("vgpr_count", 0))
        waves = min(8, 512 // max(8, (regs + 7) // 8 * 8)) if regs else 8
        # LDS: a 256-thread block puts one wave on each SIMD of a CU (160 KB)
        lds = int(k.get("group_segment_fixed_size", 0))
        lds_waves = min(8, 163840 // lds) if lds else 8
        for f in FIELDS:
            if f[1:] in k:
                rep.append("  %s: %s" % (f[1:], k[f[1:]]))
        rep.append("  waves per SIMD: %d (VGPR-bound %d, LDS-bound %d)" % (min(waves, lds_waves), waves, lds_waves))
    text = "\n".join(rep) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text)


if __name__ == "__main__":
    main()
