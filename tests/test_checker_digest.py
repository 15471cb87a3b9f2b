"""The CPU checker's row digest (oracle/cpuvm.cc gkcpu_sweep_digest) against
the oracle's rows, per bench configuration.  The GPU scale tests
(tests/test_gpu_scale.py) compare the device's full output with this digest,
so the checker itself must print every details form the device emits: config
3's k8sallowedlabelregex / annotation templates emit `{"label": key}` as a
one-member details object (VF_DET_KV, common.h), configs 2 and 4 set-valued
details (VF_DET_VAL) and plain `{}`."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CODE = r'''
import json, sys
sys.path[:0] = [%r, %r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, augmented_review
from oracle import cpu_baseline
from parity import oracle_for, oracle_review
cfg, n = int(sys.argv[1]), int(sys.argv[2])
ts, cs = getattr(W, "config%%d" %% cfg)()
gen = {2: lambda: W.gen_pods_json(n, seed=42, n_namespaces=50, start=0),
       3: lambda: W.gen_config3_json(n, seed=7, start=0),
       4: lambda: W.gen_config4_json(n, seed=1234, start=0)}[cfg]
objs, nss = gen()
objs = [json.loads(o) for o in objs]
nss = [json.loads(x) if x else None for x in nss]
d = gkgpu.Driver(host_only=True); cl = Client(d)
for t in ts: cl.add_template(t)
for c in cs: cl.add_constraint(c)
got = cpu_baseline.sweep_digest(d, d.stage_objects(objs, nss), threads=4)
od = oracle_for(ts, cs)
cidx = {kn: i for i, kn in enumerate(d.constraints())}
rows = []
kv = 0
for i, (o, ns) in enumerate(zip(objs, nss)):
    for kind, name, msg, det, _ea in oracle_review(od, augmented_review(o, ns)):
        rows.append((i, cidx[(kind, name)], msg, det))
        kv += det.startswith('{"label"')
print(json.dumps([got[1], got[2], got[3], cpu_baseline.row_digest(rows), len(rows), kv]))
''' % (os.path.join(ROOT, "gatekeeper-1_amd"), ROOT, os.path.join(ROOT, "tests"))


@pytest.mark.parametrize("cfg,n", [(2, 400), (3, 600), (4, 500)])
def test_checker_digest_equals_oracle_rows(cfg, n):
    out = subprocess.run([sys.executable, "-c", CODE, str(cfg), str(n)], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    v, fl, dg, wd, wn, kv = json.loads(out.stdout.strip().splitlines()[-1])
    assert fl == 0 and v == wn > 50, (cfg, v, wn, fl)
    if cfg == 3:
        assert kv > 20, kv  # the one-member details form is exercised
    assert dg == wd, (cfg, "checker row digest differs from the oracle's")
