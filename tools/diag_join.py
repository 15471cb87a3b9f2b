"""Diagnostic: tests/test_joins.py's edge-key join on the device, printing the
fallback reasons of flagged reviews and the label value types behind them."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "gatekeeper-1_amd")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
import test_joins as T  # noqa: E402
from parity import run_objects  # noqa: E402
from gkgpu.client import data_path  # noqa: E402

vals = ["a", "b", 7, 7.0, True, None, {"x": 1}, "a", 3, False]
objs = T._labelled(120, 5, value=lambda r, i: vals[r.randint(0, len(vals) - 1)])
cs = [W.constraint("K8sJoinLabelParam", "c", parameters={"label": "app"})]
extra = [(data_path(o), o) for o in objs]
drv = gkgpu.Driver(jit=os.environ.get("DIAG_JIT", "1") == "1")
rep, res = run_objects(drv, [T.LABEL_PARAM], cs, objs, T._ns(objs), extra_data=extra)
print("report", rep)
c = collections.Counter()
for i, o in enumerate(objs):
    if res.status[i]:
        v = o["spec"]["tags"].get("app", "<none>")
        c[(res.status[i], res.reason[i], type(v).__name__)] += 1
for k, n in sorted(c.items(), key=str):
    print("flagged status/reason/type", k, n)
