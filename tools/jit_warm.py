"""Compile the template kernels of the bench configurations with hipRTC on
the host (no GPU needed: gfx950 is an explicit offload target) into the
tree's .jitcache, so a GPU box starts with the code objects the driver's runs
need.  Kernel sources are keyed by their text (jit.cc jit_compile), so a
stale entry is simply never read.

    python tools/jit_warm.py [--configs 1,2,3,4,5,6]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gatekeeper-1_amd"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,4,5,6")
    a = ap.parse_args()
    os.environ.setdefault("GKGPU_JIT_CACHE", os.path.join(ROOT, ".jitcache"))
    os.makedirs(os.environ["GKGPU_JIT_CACHE"], exist_ok=True)
    import gkgpu
    from gkgpu import workloads as W
    from gkgpu.client import Client
    for cfg in [int(x) for x in a.configs.split(",") if x]:
        ts, cs = getattr(W, "config%d" % cfg)()
        d = gkgpu.Driver(host_only=True)
        cl = Client(d)
        for t in ts:
            cl.add_template(t)
        for c in cs:
            cl.add_constraint(c)
        t0 = time.time()
        for t in ts:
            k = t["spec"]["crd"]["spec"]["names"]["kind"]
            print("config %d %s %s" % (cfg, k, d.template_backend(k)), flush=True)
        print("config %d: %.1f s" % (cfg, time.time() - t0), flush=True)


if __name__ == "__main__":
    main()
