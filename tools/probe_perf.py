"""GPU probe: per-constraint kernel time and VM step statistics (GKGPU_PROFILE=1)."""
import os
import sys
import time

os.environ.setdefault("GKGPU_PROFILE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
ts, cs = W.config2()
objs, nss = W.gen_pods_json(N, seed=42, n_namespaces=1000)
sets = [[c] for c in cs] + [cs]
for sel in sets:
    d = gkgpu.Driver(jit=os.environ.get("GKGPU_JIT", "1") != "0")
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in sel:
        cl.add_constraint(c)
    b = d.stage_objects(objs, nss)
    b.eval(decode=False, light=True)
    t0 = time.perf_counter()
    r = b.eval(decode=False, light=True)
    wall = (time.perf_counter() - t0) * 1e3
    name = "+".join(c["kind"] for c in sel)
    print("%-60s kernel %.2f ms wall %.2f ms tuples %d launches %s" % (name[:60], r.timing_ms[2], wall, r.device_tuples,
                                                                       [(k, round(ms, 2), n) for k, ms, n in r.launches]))
    for i, (sm, mx, lanes, wmax) in enumerate(r.vm_stats()):
        waves = (N + 63) // 64
        print("   c%d steps/lane %.1f max %d lanes %d  wave-max avg %.1f  (SIMD efficiency %.2f)" % (
            i, sm / max(lanes, 1), mx, lanes, wmax / waves, (sm / 64) / max(wmax, 1)))
    b.free()
    d.close()
