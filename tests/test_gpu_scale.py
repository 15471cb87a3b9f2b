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


def _run(cfg, n, gen, max_fallback_frac):
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
    od = oracle_for(ts, cs)
    reviews = [augmented_review(json.loads(objs[i]), None if nss[i] is None else json.loads(nss[i])) for i in sample]
    rep = compare(od, reviews, sub)
    print("config %d sample:" % cfg, rep, "heaviest lane emitted", int(counts.max()), flush=True)
    assert not rep.mismatches, rep.mismatches[:3]
    assert rep.compared >= N_SAMPLE - 64 - 2 * flagged
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
