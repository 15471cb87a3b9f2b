"""Parity at benchmark size: the bench's own
workloads -- config 2 (1M Pods x the 5 agilebank constraints) and config 4
(1.25M mixed resources x 50 randomized constraints, one GPU's shard of the 10M
sweep) -- staged and evaluated on the GPU exactly as bench.py does, then:

  * ORACLE PARITY on a stratified sample of >= 2,000 reviews: every review
    whose lane emitted the most tuples (the lane-capacity edge), the first
    and last 64 reviews of the batch, and an even spread over the whole batch
    (one review per stratum).  The sampled reviews' rows are picked out of the
    device output on the GPU (gk_results_copy_device_output: the raw gk_viol
    records and message bytes) and compared with the CPU oracle's (tests/
    parity.py compare: multisets of (constraint, msg, details, action)).
  * Every flagged review (error / CPU fallback) is counted and must be rare;
    flagged reviews in the sample must be flagged because the oracle errors
    (error) or are excluded (fallback), as compare() checks.
  * FULL POPULATION against the CPU checker: an order-free digest of EVERY
    row of the device output -- (review, constraint, message bytes, details
    bytes), oracle/cpuvm.cc gkcpu_rows_digest -- equals the digest of the rows
    the host build of the same programs produces over the same staged batch
    (gkcpu_sweep_digest).  The host compiler is independent of the device
    compiler, so a device miscompile or a lost / duplicated / corrupted row
    anywhere in the 1M reviews shows here, not only in the sample.  (The
    checker's rows themselves are pinned to the oracle's by
    tests/test_checker_digest.py.)
  * SELF-CONSISTENCY (not parity): the audit sweep's exact totals
    (Batch.eval_audit, device sampling) equal the per-constraint counts of the
    decoded device output.
"""
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu

N_SAMPLE = 2000


def _run(cfg, n, gen, max_fallback_frac, inventory=(), oracle_factory=None):
    import torch
    import gkgpu
    from gkgpu import workloads as W
    from gkgpu.client import Client, augmented_review
    from gkgpu.driver import Result, Results
    from gkgpu.page import Page
    from gkgpu.parallel import DeviceOutput, unpack_viol
    from parity import compare, oracle_for
    if not gkgpu.Driver.device_available():
        pytest.fail("no HIP device visible")
    ts, cs = getattr(W, "config%d" % cfg)()
    objs, nss = gen(n)
    drv = gkgpu.Driver()
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    for path, js in inventory:
        drv.put_data(path, json.loads(js))
    batch = drv.stage_page(Page.from_lists(objs, nss))
    dev = torch.device("cuda", 0)
    dout = DeviceOutput(dev)
    res = batch.eval(decode=False, light=True, device_out=dout, with_status=True)
    status = res.status
    flagged = int((status & 3).astype(bool).sum()) if len(status) else 0
    print("config %d: %d reviews, %d tuples, %d flagged" % (cfg, n, res.device_tuples, flagged), flush=True)
    assert flagged <= max_fallback_frac * n, flagged
    tup = dout.tuples()
    # per-review emission counts -> the heaviest lanes
    counts = torch.bincount(tup[:, 0].long(), minlength=n)
    heavy = torch.topk(counts, 64).indices.cpu().tolist()
    rng = random.Random(cfg)
    strata = N_SAMPLE - 64 - 128
    spread = [min(n - 1, (k * n) // strata + rng.randrange(max(1, n // strata))) for k in range(strata)]
    sample = sorted(set(heavy) | set(range(64)) | set(range(n - 64, n)) | set(spread))
    assert len(sample) >= N_SAMPLE - 64, len(sample)
    idx = torch.tensor(sample, dtype=torch.int32, device=dev)
    sel = tup[torch.isin(tup[:, 0], idx)].cpu().numpy()
    raw = dout.bytes()
    cons = drv.constraints()
    ea = {(c["kind"], c["metadata"]["name"]): c.get("spec", {}).get("enforcementAction", "deny") for c in cs}
    pos = {r: k for k, r in enumerate(sample)}
    rows = []
    for rec in sel:
        rv, c, seq, rule, ml, mo, dl = unpack_viol(rec)
        b = raw[mo:mo + ml + dl].cpu().numpy().tobytes()
        kind, name = cons[c]
        rows.append(Result(pos[rv], c, kind, name, b[:ml].decode("utf-8", "surrogateescape"),
                           b[ml:].decode("utf-8", "surrogateescape"), ea[(kind, name)]))
    sub = Results(rows, [int(status[i]) if len(status) else 0 for i in sample], [0] * len(sample), [])
    od = oracle_factory(ts, cs) if oracle_factory else oracle_for(ts, cs)
    reviews = [augmented_review(json.loads(objs[i]), None if nss[i] is None else json.loads(nss[i])) for i in sample]
    rep = compare(od, reviews, sub)
    print("config %d sample:" % cfg, rep, "heaviest lane emitted", int(counts.max()), flush=True)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.canonical_only == 0, rep  # byte-exact rows (no object-printing template here)
    assert rep.compared >= N_SAMPLE - 64 - 2 * flagged
    # full population: every row against the CPU checker's
    from oracle import cpu_baseline
    gd, gn = cpu_baseline.device_rows_digest(tup.cpu().numpy(), raw.cpu().numpy(), threads=16)
    ev, cn, cfl, cd = cpu_baseline.sweep_digest(drv, batch, threads=16)
    print("config %d full population: device rows %d, checker rows %d, checker flagged pairs %d" % (cfg, gn, cn, cfl),
          flush=True)
    assert flagged == 0 and cfl == 0, (flagged, cfl)
    assert gn == cn and gn == len(tup), (gn, cn, len(tup))
    assert gd == cd, "config %d: the device rows differ from the CPU checker's" % cfg
    # self-consistency: the audit sweep's totals vs the decoded output's counts
    sweep = batch.eval_audit(limit=20)
    if not len(status) or not (status & 3).any():
        per_c = torch.bincount(tup[:, 1].long(), minlength=len(cons)).cpu().tolist()
        assert [int(x) for x in sweep.totals] == per_c
    return rep


def test_config2_bench_workload_parity_at_1m():
    from gkgpu import workloads as W
    _run(2, 1_000_000, lambda n: W.gen_pods_json(n, seed=42, n_namespaces=1000, start=0), 0.0)


def test_config4_bench_workload_parity_at_1_25m():
    from gkgpu import workloads as W
    _run(4, 1_250_000, lambda n: W.gen_config4_json(n, seed=1234, start=0), 0.01)


def test_config3_bench_workload_parity_at_1m():
    """config 3: 1M Deployments + Services x the 10 allowedRegex constraints"""
    from gkgpu import workloads as W
    _run(3, 1_000_000, lambda n: W.gen_config3_json(n, seed=7, start=0), 0.0)


class _KeyGroupOracle:
    """The oracle for config 6 at 200K synced objects.  Scanning the whole
    inventory per review (what topdown does for unique-label /
    unique-service-selector) is out of reach for the Python restatement at
    this size, so per sampled review the oracle's data.inventory holds every
    synced object whose JSON carries the review's own `app` value as a string
    token -- a superset of the objects whose label value / flattened selector
    can equal the review's, the only ones the templates' equality literal lets
    produce a row (k8suniquelabel_template.yaml:49-55,
    k8suniqueserviceselector_template.yaml:40-46) -- plus 24 objects of other
    keys.  The device evaluated against all 200K."""

    def __init__(self, od, inventory, seed=6):
        import re
        self.od = od
        self.app = re.compile(r'"app":"(app-[0-9]+)"')
        self.groups = {}
        for path, js in inventory:
            for a in set(self.app.findall(js)):
                self.groups.setdefault(a, []).append((path, js))
        self.inv = inventory
        self.rng = random.Random(seed)

    def query(self, path, input_json):
        rv = json.loads(input_json)["review"]
        obj = rv.get("object") or {}
        a = ((obj.get("metadata") or {}).get("labels") or {}).get("app") or \
            ((obj.get("spec") or {}).get("selector") or {}).get("app")
        put = list(self.groups.get(a, [])) if isinstance(a, str) else []
        put += [self.inv[self.rng.randrange(len(self.inv))] for _ in range(24)]
        seen = set()
        put = [(p, js) for p, js in put if not (p in seen or seen.add(p))]
        for p, js in put:
            self.od.put_data(p, js)
        try:
            return self.od.query(path, input_json)
        finally:
            for p, _ in put:
                self.od.delete_data(p)


def test_config6_bench_workload_parity_at_200k():
    """config 6: the agilebank constraints + unique-label over 200K objects
    that are also the synced inventory (the bench's join workload); the
    stratified sample against the key-group oracle above"""
    from gkgpu import workloads as W
    from parity import oracle_for
    objs, nss = W.gen_config6_json(200_000)
    inv = W.inventory_paths(objs)
    rep = _run(6, len(objs), lambda n: (objs, nss), 0.0, inventory=inv,
               oracle_factory=lambda ts, cs: _KeyGroupOracle(oracle_for(ts, cs), inv))
    assert rep.violations > 200, rep
