"""Multi-rank audit on real engine shards: two gloo ranks share
cuda:0, each stages its own contiguous shard of config-2 Pods through the
engine, sweeps it on the GPU (Batch.eval_audit) and runs the audit exchange
(gkgpu/parallel.py exchange_audit: int64 totals all-reduce + first-`limit`
samples gathered to rank 0).  Rank 0 checks the merged statuses against
  * a single-process sweep of the union (one engine, one batch), and
  * the CPU oracle's statuses of the union (pkg/audit/manager.go:462-508 over
    the oracle's per-object results, tests/parity.py),
which must all be identical.  The RCCL leg of the same code runs only on the
driver's multi-GPU node; everything around it is pinned here."""
import os
import socket

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


PER, LIMIT, NS = 700, 20, 40


def _shard(rank):
    from gkgpu import workloads as W
    return W.gen_pods_json(PER, seed=42, n_namespaces=NS, start=rank * PER)


def _engine():
    import gkgpu
    from gkgpu import workloads as W
    from gkgpu.client import Client
    ts, cs = W.config2()
    drv = gkgpu.Driver(device=0)
    cl = Client(drv)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    return drv, ts, cs


def _rank(rank, world, port, q):
    import sys
    sys.path[:0] = [HERE, ROOT, os.path.join(ROOT, "gatekeeper-1_amd")]
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch  # noqa: F401  (one HIP runtime: torch first, gkgpu.driver)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gkgpu.audit import AuditWriter
        from gkgpu.page import Page
        from gkgpu.parallel import exchange_audit
        drv, ts, cs = _engine()
        objs, nss = _shard(rank)
        batch = drv.stage_page(Page.from_lists(objs, nss))
        cons = drv.constraints()

        def res_of(b):
            return lambda i: b.resource(i)[1:]

        sweep = batch.eval_audit(limit=LIMIT)
        merged = exchange_audit(sweep, rank * PER, res_of(batch), cons, limit=LIMIT, dst=0)
        if rank == 0:
            # one process, one batch over the union
            all_objs, all_nss = [], []
            for r in range(world):
                o, n = _shard(r)
                all_objs += o
                all_nss += n
            whole = drv.stage_page(Page.from_lists(all_objs, all_nss))
            single = AuditWriter.from_sweep(cons, whole.eval_audit(limit=LIMIT), res_of(whole), LIMIT)
            # the oracle over the union, in evaluation order
            import json
            from gkgpu.client import augmented_review
            from parity import oracle_for, oracle_review
            od = oracle_for(ts, cs)
            cidx = {k: i for i, k in enumerate(cons)}
            oracle = AuditWriter(cons, LIMIT)
            for o, n in zip(all_objs, all_nss):
                obj = json.loads(o)
                rows = oracle_review(od, augmented_review(obj, json.loads(n) if n else None))
                assert rows != "ERROR"
                for kind, name, msg, _det, ea in rows:
                    md = obj["metadata"]
                    oracle.add(cidx[(kind, name)], (obj["kind"], md["name"], md.get("namespace", "")), msg, ea)
            q.put(("ok", merged.statuses() == single.statuses(), merged.statuses() == oracle.statuses(),
                   merged.per_action == oracle.per_action, sum(merged.totals.values()), sweep.n_fallbacks))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put(("err", traceback.format_exc(), None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_engine_shards_exchange_on_one_gpu():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env_keep = dict(os.environ)
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        status, same_single, same_oracle, same_actions, total, fb = q.get(timeout=280)
    finally:
        for p in ps:
            p.join(60)
            if p.is_alive():
                p.kill()
    os.environ.clear()
    os.environ.update(env_keep)
    assert status == "ok", same_single
    assert fb == 0
    assert same_single, "merged shard statuses differ from one sweep over the union"
    assert same_oracle, "merged shard statuses differ from the oracle's"
    assert same_actions and total > 1000
