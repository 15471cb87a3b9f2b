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
