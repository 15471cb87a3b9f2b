"""Step-by-step GPU diagnostic (prints after every driver call; dumps the
Python stack if a step hangs).  python tools/diag_r03.py [n]"""
import faulthandler
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
faulthandler.dump_traceback_later(100, exit=True)

t0 = time.time()


def say(*a):
    print("[%7.2f]" % (time.time() - t0), *a, flush=True)


import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402

say("device_available", gkgpu.Driver.device_available())
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
for jit in (False, True):
    ts, cs = W.config1()
    nss = W.gen_namespaces(n, seed=1)
    d = gkgpu.Driver(jit=jit)
    from parity import engine_for, oracle_for, run_objects  # noqa: E402
    engine_for(d, ts, cs)
    say("jit", jit, "engine ready")
    k = ts[0]["spec"]["crd"]["spec"]["names"]["kind"]
    say("backend", d.template_backend(k))
    res = d.review_objects(nss, [None] * len(nss))
    say("review_objects", len(res.results), "timing", res.timing_ms)
    rep, res = run_objects(gkgpu.Driver(jit=jit), ts, cs, nss, [None] * len(nss))
    say("parity", rep)
    ts, cs = W.config2()
    pods, ns_of, ns_objs = W.gen_pods(n, seed=42, n_namespaces=20)
    rep, res = run_objects(gkgpu.Driver(jit=jit), ts, cs, pods, [ns_objs[x] for x in ns_of])
    say("config2 parity", rep)
say("done")
