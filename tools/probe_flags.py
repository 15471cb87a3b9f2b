"""GPU probe: flagged reviews (error / CPU fallback) of a staged config at full
size, with their reason codes and the constraints / kinds involved."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402
from gkgpu.page import Page  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "4"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_250_000
ts, cs = {"2": W.config2, "3": W.config3, "4": W.config4}[cfg]()
gen = {"2": lambda: W.gen_pods_json(n, seed=42, n_namespaces=1000), "3": lambda: W.gen_config3_json(n, seed=7),
       "4": lambda: W.gen_config4_json(n, seed=1234)}[cfg]
objs, nss = gen()
d = gkgpu.Driver()
cl = Client(d)
for t in ts:
    cl.add_template(t)
for c in cs:
    cl.add_constraint(c)
b = d.stage_page(Page.from_lists(objs, nss))
for k in range(3):  # repeated sweeps of one staged batch (bench.py's steps)
    a = b.eval_audit(limit=20)
    print("sweep %d: errors %d fallbacks %d" % (k, a.n_errors, a.n_fallbacks), flush=True)
import ctypes as C  # noqa: E402
import json  # noqa: E402
import numpy as np  # noqa: E402
lib = d._lib
out = C.c_void_p()
d._check(lib.gk_batch_eval(d._e, b._h, 0, C.byref(out)))
nr = lib.gk_results_reviews(out)
st = np.zeros(max(nr, 1), dtype=np.uint32)
rs = np.zeros(max(nr, 1), dtype=np.uint32)
lib.gk_results_copy_status(out, st.ctypes.data, rs.ctypes.data)
lib.gk_results_free(out)
fl = np.nonzero(st[:nr] & 3)[0]
print("config %s n %d flagged %d (error %d, fallback %d)" % (cfg, n, len(fl), int((st & 1).astype(bool).sum()),
                                                             int((st & 2).astype(bool).sum())), flush=True)
if len(fl):
    print("reasons", collections.Counter(rs[fl].tolist()), "status", collections.Counter(st[fl].tolist()))
    print("kinds", collections.Counter(json.loads(objs[i])["kind"] for i in fl))
    print("example", objs[fl[0]][:800])
