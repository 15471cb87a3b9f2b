"""Multi-rank path on CPU: world_size-2 gloo runs of the violation gather and
the totals all-reduce (gkgpu/parallel.py), the same code the RCCL ranks run."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gkgpu.parallel import Gatherer, decode, pack_viol, shard_range, unpack_viol, VIOL_WORDS


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_output(rank, n_reviews):
    """synthetic per-rank engine output: reviews get rank-dependent violations"""
    msgs, rows = bytearray(), []
    for rv in range(n_reviews):
        for seq in range((rv + rank) % 3):
            m = ("r%d-review%d-v%d" % (rank, rv, seq)).encode()
            d = b"{}"
            rows.append(pack_viol(rv, (rv + seq) % 2, seq, 0, len(m), len(msgs), len(d)))
            msgs += m + d
    t = torch.tensor(rows, dtype=torch.int32).view(-1, VIOL_WORDS) if rows else torch.zeros((0, VIOL_WORDS), dtype=torch.int32)
    # shuffle: the device output order is one reservation per wavefront
    g = torch.Generator().manual_seed(rank)
    t = t[torch.randperm(t.shape[0], generator=g)]
    return t, torch.tensor(list(msgs), dtype=torch.uint8)


def _worker(rank, world, port, n_total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lo, hi = shard_range(n_total, rank, world)
        t, b = _rank_output(rank, hi - lo)
        totals = torch.zeros(2, dtype=torch.int64)
        for c in t[:, 1].tolist():
            totals[c] += 1
        dist.all_reduce(totals)
        g = Gatherer(dst=0)
        for _ in range(2):  # steady state reuses the receive buffers
            parts = g.gather(t, b, review_base=lo)
        if rank == 0:
            q.put(("ok", decode(parts), totals.tolist()))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [10, 7])
def test_gather_two_ranks_gloo(n_total):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in ps:
        p.start()
    status, rows, totals = q.get(timeout=120)
    for p in ps:
        p.join(60)
    assert status == "ok", rows
    # expected: every rank's rows, review indices rebased to global, in reference order
    want = []
    for r in range(world):
        lo, hi = shard_range(n_total, r, world)
        t, b = _rank_output(r, hi - lo)
        bb = bytes(b.tolist())
        for rec in t.tolist():
            rv, c, seq, rule, ml, mo, dl = unpack_viol(rec)
            do = mo + ml
            want.append((rv + lo, c, seq, rule, bb[mo:mo + ml].decode(), bb[do:do + dl].decode()))
    want.sort(key=lambda x: (x[0], x[1], x[2]))
    assert rows == want
    assert sum(totals) == len(want)
    assert totals == [sum(1 for w in want if w[1] == c) for c in range(2)]


def test_shard_range_covers_exactly():
    for n in (0, 1, 7, 10, 1001):
        for world in (1, 2, 3, 8):
            got = [shard_range(n, r, world) for r in range(world)]
            flat = [i for lo, hi in got for i in range(lo, hi)]
            assert flat == list(range(n))


# -- the audit exchange (totals all-reduce + first-limit samples, gkgpu/parallel.py exchange_audit)

def _oracle_rows(n_pods=240):
    """per review: [(constraint index, autoreject?, seq, msg, enforcementAction)] from the CPU oracle"""
    import json as _json
    from gkgpu import workloads as W
    from gkgpu.client import augmented_review
    from parity import oracle_for, oracle_review
    ts, cs = W.config2()
    cs = [dict(c) for c in cs]
    cs[3] = W.constraint("K8sRequiredProbes", "must-have-probes", match=cs[3]["spec"]["match"],
                         parameters=cs[3]["spec"]["parameters"], enforcement_action="dryrun")
    od = oracle_for(ts, cs)
    pods, ns_of, ns_objs = W.gen_pods(n_pods, seed=23, n_namespaces=12)
    cidx = {(c["kind"], c["metadata"]["name"]): i for i, c in enumerate(cs)}
    per = []
    for p, n in zip(pods, ns_of):
        rows, seq = [], {}
        for kind, name, msg, _det, ea in oracle_review(od, augmented_review(p, ns_objs[n])):
            c = cidx[(kind, name)]
            rows.append((c, 1, seq.get(c, 0), msg, ea))
            seq[c] = seq.get(c, 0) + 1
        per.append(rows)
    cons = [(c["kind"], c["metadata"]["name"]) for c in cs]
    actions = [c.get("spec", {}).get("enforcementAction", "deny") for c in cs]
    res = [("Pod", p["metadata"]["name"], p["metadata"]["namespace"]) for p in pods]
    return per, cons, actions, res


def _sweep_of(per, lo, hi, ncons, actions, limit):
    """an engine-shaped AuditSweep for reviews [lo, hi) (local review indices)"""
    from gkgpu.driver import AuditSweep, Sample
    totals = [0] * ncons
    cand = []
    for r in range(lo, hi):
        for c, ar, seq, msg, ea in per[r]:
            totals[c] += 1
            cand.append((c, r - lo, ar, seq, msg, ea))
    cand.sort(key=lambda x: (x[0], x[1], x[2], x[3]))
    samples, taken = [], {}
    for c, rv, ar, seq, msg, ea in cand:
        if taken.get(c, 0) < limit:
            taken[c] = taken.get(c, 0) + 1
            b = msg.encode()
            samples.append(Sample(rv, c, seq, 0 if ar else 0xffff, len(b), b[:256], ea))
    return AuditSweep(totals, samples, actions, 0, 0, 0, [], 0, 0, [])


def _audit_worker(rank, world, port, limit, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "gatekeeper-1_amd")]
        from gkgpu.audit import AuditWriter
        from gkgpu.parallel import exchange_audit
        per, cons, actions, res = _oracle_rows()
        lo, hi = shard_range(len(per), rank, world)
        sweep = _sweep_of(per, lo, hi, len(cons), actions, limit)
        merged = exchange_audit(sweep, lo, lambda i: res[lo + i], cons, limit=limit)
        if rank == 0:
            single = AuditWriter(cons, limit)
            for r, rows in enumerate(per):
                for c, _ar, _seq, msg, ea in rows:
                    single.add(c, res[r], msg, ea)
            q.put(("ok", merged.statuses() == single.statuses(), merged.per_action == single.per_action,
                   sum(merged.totals.values())))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put(("err", traceback.format_exc(), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,limit", [(2, 3), (2, 20), (3, 5)])
def test_audit_exchange_equals_single_process_sweep(world, limit):
    """shards' engine-shaped sweeps, exchanged over gloo, give exactly the
    statuses of one sweep over all resources (manager.go:462-508)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_audit_worker, args=(r, world, port, limit, q)) for r in range(world)]
    for p in ps:
        p.start()
    status, same, same_act, total = q.get(timeout=240)
    for p in ps:
        p.join(60)
    assert status == "ok", same
    assert same and same_act and total > 100


# -- flagged reviews (GK_REVIEW_ERROR / GK_REVIEW_FALLBACK): ADVICE r02.  The
# engine leaves them out of totals and samples; the caller's CPU driver answers
# them and the status writer merges them in at their place in evaluation order.

def _flagged_sweep(per, lo, hi, ncons, actions, limit, flagged):
    """_sweep_of with the reviews `flagged` (local indices) removed, as the
    engine reports them"""
    keep = [rows if (r - lo) not in flagged else [] for r, rows in enumerate(per[lo:hi], start=lo)]
    full = list(per)
    full[lo:hi] = keep
    sw = _sweep_of(full, lo, hi, ncons, actions, limit)
    sw.flagged = sorted(flagged)
    return sw


def test_from_sweep_merges_flagged_reviews():
    from gkgpu.audit import AuditWriter, FlaggedReviews
    per, cons, actions, res = _oracle_rows(120)
    flagged = {0, 3, 17, 50, 119}
    sweep = _flagged_sweep(per, 0, len(per), len(cons), actions, 5, flagged)
    with pytest.raises(FlaggedReviews):
        AuditWriter.from_sweep(cons, sweep, lambda i: res[i], 5)
    fb = lambda i: [(c, msg, ea) for c, _ar, _seq, msg, ea in per[i]]  # noqa: E731  (the CPU driver)
    got = AuditWriter.from_sweep(cons, sweep, lambda i: res[i], 5, fallback=fb)
    want = AuditWriter(cons, 5)
    for r, rows in enumerate(per):
        for c, _ar, _seq, msg, ea in rows:
            want.add(c, res[r], msg, ea)
    assert got.statuses() == want.statuses()
    assert got.per_action == want.per_action


def _flagged_worker(rank, world, port, limit, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "gatekeeper-1_amd")]
        from gkgpu.audit import AuditWriter
        from gkgpu.parallel import exchange_audit
        per, cons, actions, res = _oracle_rows()
        lo, hi = shard_range(len(per), rank, world)
        flagged = {i for i in range(hi - lo) if (i * 7 + rank) % 11 == 0}
        sweep = _flagged_sweep(per, lo, hi, len(cons), actions, limit, flagged)
        fb = lambda i: [(c, msg, ea) for c, _ar, _seq, msg, ea in per[lo + i]]  # noqa: E731
        merged = exchange_audit(sweep, lo, lambda i: res[lo + i], cons, limit=limit, fallback=fb)
        if rank == 0:
            single = AuditWriter(cons, limit)
            for r, rows in enumerate(per):
                for c, _ar, _seq, msg, ea in rows:
                    single.add(c, res[r], msg, ea)
            q.put(("ok", merged.statuses() == single.statuses(), merged.per_action == single.per_action,
                   sum(merged.totals.values())))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put(("err", traceback.format_exc(), None, None))
        raise
    finally:
        dist.destroy_process_group()


def test_audit_exchange_merges_flagged_reviews():
    """each rank answers its flagged reviews through the fallback before the
    exchange: the merged statuses equal one sweep's over all resources"""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_flagged_worker, args=(r, world, port, 4, q)) for r in range(world)]
    for p in ps:
        p.start()
    status, same, same_act, total = q.get(timeout=240)
    for p in ps:
        p.join(60)
    assert status == "ok", same
    assert same and same_act and total > 100


def _one_flagged_worker(rank, world, port, q):
    """only rank 1 holds flagged reviews and nobody passes a fallback: every
    rank must raise FlaggedReviews (none may wait in a collective)"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        here = os.path.dirname(os.path.abspath(__file__))
        sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "gatekeeper-1_amd")]
        from gkgpu.audit import FlaggedReviews
        from gkgpu.parallel import exchange_audit
        per, cons, actions, res = _oracle_rows(60)
        lo, hi = shard_range(len(per), rank, world)
        flagged = {2, 5} if rank == 1 else set()
        sweep = _flagged_sweep(per, lo, hi, len(cons), actions, 4, flagged)
        try:
            exchange_audit(sweep, lo, lambda i: res[lo + i], cons, limit=4)
            q.put((rank, "returned"))
        except FlaggedReviews as ex:
            q.put((rank, "raised: " + str(ex)))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, "err " + traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def test_audit_exchange_flagged_on_one_rank_raises_everywhere():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_one_flagged_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(60)
    assert got[1].startswith("raised: 2 reviews flagged"), got
    assert got[0].startswith("raised: 1 peer rank"), got
