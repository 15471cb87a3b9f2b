"""Multi-GPU audit sweep: resource shards per rank, violations gathered to rank 0.

SURVEY 8(e): resources are independent units, so each rank (one process per
GPU) audits a contiguous shard of the resources against every constraint with
no data-path collective.  The exchange steps are the ones the audit needs
downstream: the per-constraint totals (an all-reduce, the status write of
pkg/audit/manager.go:462-508) and the compacted violation lists, gathered to
rank 0 with exact-size point-to-point transfers over RCCL (xGMI) -- or gloo
for the CPU tests.

The violation records are the engine's gk_viol (include/gkgpu.h), 32 bytes:
u32 review, u32 constraint, u16 seq, u16 rule, u32 msg_len, u64 msg_off,
u32 det_len, u32 pad (details JSON follows the message).  Viewed as 8 int32
words: [review, constraint, seq | rule << 16, msg_len, off_lo, off_hi,
det_len, pad].  A rank's review indices are rebased to global indices before
sending; message offsets stay relative to that rank's byte buffer, so rank 0
holds one (tuples, bytes) pair per source rank.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

VIOL_WORDS = 8
VIOL_BYTES = 32


def pack_viol(review, constraint, seq, rule, msg_len, msg_off, det_len):
    """one gk_viol record as 8 int32 words (two's complement)"""
    def i32(x):
        x &= 0xffffffff
        return x - (1 << 32) if x >= 1 << 31 else x
    return [i32(review), i32(constraint), i32(seq | (rule << 16)), i32(msg_len), i32(msg_off), i32(msg_off >> 32),
            i32(det_len), 0]


def unpack_viol(words):
    """(review, constraint, seq, rule, msg_len, msg_off, det_len) of 8 int32 words"""
    w = [int(x) & 0xffffffff for x in words]
    return w[0], w[1], w[2] & 0xffff, w[2] >> 16, w[3], w[4] | (w[5] << 32), w[6]


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard [start, stop) of n_total resources for `rank`: ceil(n/world) each."""
    per = (n_total + world - 1) // world
    start = min(n_total, rank * per)
    return start, min(n_total, start + per)


def _global_rank(group):
    """group rank -> the global rank torch.distributed.P2POp expects as its peer
    (ranks are group-local everywhere else; identity for the default group)"""
    import torch.distributed as dist
    if group is None:
        return lambda r: r
    return lambda r: dist.get_global_rank(group, r)


class DeviceOutput:
    """Reusable device buffers receiving one evaluation's raw output
    (Batch.eval(device_out=...)); grown on demand, kept across steps."""

    def __init__(self, device):
        import torch
        self.torch = torch
        self.device = device
        self._t = None
        self._b = None
        self.n_tuples = 0
        self.n_bytes = 0

    def __call__(self, n_tuples: int, n_bytes: int):
        torch = self.torch
        if self._t is None or self._t.numel() < n_tuples * VIOL_BYTES:
            self._t = torch.empty(max(n_tuples, 1) * VIOL_BYTES, dtype=torch.uint8, device=self.device)
        if self._b is None or self._b.numel() < n_bytes:
            self._b = torch.empty(max(n_bytes, 1), dtype=torch.uint8, device=self.device)
        self.n_tuples, self.n_bytes = n_tuples, n_bytes
        return self._t.data_ptr(), self._b.data_ptr()

    def copied(self, n_tuples: int):
        """records actually written (the engine drops those of flagged reviews)"""
        self.n_tuples = n_tuples

    def tuples(self):
        """int32 [n, 8] view of the gk_viol records."""
        return self._t[: self.n_tuples * VIOL_BYTES].view(self.torch.int32).view(-1, VIOL_WORDS)

    def bytes(self):
        return self._b[: self.n_bytes]


class Gatherer:
    """Gathers every rank's violation tuples and message bytes to `dst`.

    Receive buffers on `dst` are kept across calls (an audit sweep repeats with
    the same shapes), so a steady-state gather allocates nothing."""

    def __init__(self, dst: int = 0, group=None):
        self.dst = dst
        self.group = group
        self._recv = {}

    def gather(self, tuples, bytes_, review_base: int):
        """tuples: int32 [n, 8] (gk_viol) and bytes_: uint8 [m] on this rank's
        device (CPU tensors under gloo).  Returns, on `dst`, a list with one
        (tuples, bytes) pair per rank in rank order -- review indices global,
        byte offsets relative to that pair's bytes -- and None elsewhere."""
        import torch
        import torch.distributed as dist
        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        peer = _global_rank(self.group)
        dev = tuples.device
        t = tuples
        if review_base:
            t = tuples.clone()
            t[:, 0] += int(review_base)
        counts = torch.tensor([t.shape[0], bytes_.numel()], dtype=torch.int64, device=dev)
        allc = [torch.zeros_like(counts) for _ in range(world)]
        dist.all_gather(allc, counts, group=self.group)
        sizes = [(int(c[0]), int(c[1])) for c in allc]
        ops = []
        out: Optional[List] = None
        if rank == self.dst:
            out = []
            for r in range(world):
                nt, nb = sizes[r]
                if r == rank:
                    out.append((t, bytes_))
                    continue
                key = (r, nt, nb)
                if key not in self._recv:
                    self._recv = {k: v for k, v in self._recv.items() if k[0] != r}
                    self._recv[key] = (torch.empty((nt, VIOL_WORDS), dtype=torch.int32, device=dev),
                                       torch.empty(nb, dtype=torch.uint8, device=dev))
                rt, rb = self._recv[key]
                if nt:
                    ops.append(dist.P2POp(dist.irecv, rt, peer(r), self.group))
                if nb:
                    ops.append(dist.P2POp(dist.irecv, rb, peer(r), self.group))
                out.append((rt, rb))
        else:
            nt, nb = sizes[rank]
            if nt:
                ops.append(dist.P2POp(dist.isend, t.contiguous(), peer(self.dst), self.group))
            if nb:
                ops.append(dist.P2POp(dist.isend, bytes_.contiguous(), peer(self.dst), self.group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        return out


def decode(parts, limit: Optional[int] = None):
    """(review, constraint, seq, rule, msg, details) rows from gathered parts,
    in the reference's per-object order (review, autoreject first, constraint,
    emission order).  Host-side; for tests and status samples."""
    rows = []
    for t, b in parts:
        tt = t.cpu().numpy()
        bb = b.cpu().numpy().tobytes()
        for rec in tt:
            rv, c, seq, rule, ml, mo, dl = unpack_viol(rec)
            do = mo + ml
            rows.append((rv, 0 if rule == 0xffff else 1, c, seq, rule, bb[mo:mo + ml].decode("utf-8", "surrogateescape"),
                         bb[do:do + dl].decode("utf-8", "surrogateescape")))
    rows.sort(key=lambda r: (r[0], r[1], r[2], r[3]))
    out = [(r[0], r[2], r[3], r[4], r[5], r[6]) for r in rows]
    return out[:limit] if limit is not None else out


# ------------------------------------------------------------------ audit exchange
# after each rank's sweep, the only exchange the audit status
# needs is (i) the per-constraint totals, all-reduced as int64, and (ii) per
# constraint the first `limit` results by global resource index, which each
# rank has already selected on its device (Batch.eval_audit); rank 0 merges the
# ranks' candidates (at most constraints x limit each) and writes the statuses.
# The reference audits one object at a time in discovery order
# (manager.go:333-389), which Go map iteration makes nondeterministic; the
# engine fixes that order as the global resource index.

def _sample_rows(sweep, review_base: int, resource_of_review):
    """[global review, constraint, autoreject first (0/1), seq, msg_len, head
    (latin-1 str), enforcementAction, kind, name, namespace] per sample"""
    rows = []
    for s in sweep.samples:
        kind, name, ns = resource_of_review(s.review)
        rows.append([int(review_base) + s.review, s.constraint, 0 if s.rule == 0xffff else 1, s.seq, s.msg_len,
                     s.msg.decode("latin-1"), s.enforcement_action, kind, name, ns])
    return rows


def gather_bytes(payload: bytes, dst: int = 0, device=None, group=None):
    """every rank's payload to `dst` (list in rank order there, None elsewhere):
    an all-gather of sizes, then exact-size point-to-point transfers
    (device tensors under RCCL, CPU tensors under gloo)"""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    peer = _global_rank(group)
    dev = device if device is not None else torch.device("cpu")
    n = torch.tensor([len(payload)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(x.item()) for x in sizes]
    buf = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev) if payload else \
        torch.zeros(0, dtype=torch.uint8, device=dev)
    ops, recv = [], {}
    if rank == dst:
        for r in range(world):
            if r != rank and sizes[r]:
                recv[r] = torch.empty(sizes[r], dtype=torch.uint8, device=dev)
                ops.append(dist.P2POp(dist.irecv, recv[r], peer(r), group))
    elif sizes[rank]:
        ops.append(dist.P2POp(dist.isend, buf, peer(dst), group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != dst:
        return None
    out = []
    for r in range(world):
        if r == rank:
            out.append(payload)
        else:
            out.append(bytes(recv[r].cpu().numpy().tobytes()) if r in recv else b"")
    return out


def merge_samples(rows, limit: int):
    """first `limit` rows per constraint by (global review, autoreject first, seq)"""
    rows = sorted(rows, key=lambda r: (r[1], r[0], r[2], r[3]))
    out, cur, taken = [], None, 0
    for r in rows:
        if r[1] != cur:
            cur, taken = r[1], 0
        if taken < limit:
            out.append(r)
            taken += 1
    return out


def exchange_audit(sweep, review_base: int, resource_of_review, constraints, limit: int = 20, dst: int = 0,
                   device=None, group=None, fallback=None):
    """The multi-rank audit exchange: totals all-reduce (int64) + samples
    gathered to `dst`, merged into an AuditWriter there (None elsewhere).
    Reviews the rank's sweep flagged (error / CPU fallback) are answered by
    `fallback(i)` -> [(constraint, msg, enforcementAction)] on that rank
    before the exchange (AuditWriter.from_sweep); without one they raise --
    on every rank together: the all-reduce carries one more word, the number
    of ranks that could not answer their flagged reviews, so no rank is left
    waiting in a collective its peers never enter."""
    import json
    import torch
    import torch.distributed as dist
    from .audit import AuditWriter, FlaggedReviews, flagged_rows
    dev = device if device is not None else torch.device("cpu")
    err = None
    try:
        totals, frows = flagged_rows(sweep, fallback, review_base)
    except FlaggedReviews as ex:
        err, totals, frows = ex, [int(x) for x in sweep.totals], []
    n = max(len(constraints), len(totals))
    tot = torch.tensor(totals + [0] * (n - len(totals)) + [1 if err is not None else 0], dtype=torch.int64, device=dev)
    dist.all_reduce(tot, group=group)
    failed = int(tot[-1].item())
    if failed:
        raise err if err is not None else FlaggedReviews(
            "%d peer rank(s) hold flagged reviews without a fallback evaluator" % failed)
    tot = tot[:-1]
    rows = _sample_rows(sweep, review_base, resource_of_review)
    for rv, ar, j, c, head, ml, ea in frows:
        kind, name, ns = resource_of_review(rv - int(review_base))
        rows.append([rv, c, ar, j, ml, head.decode("latin-1"), ea, kind, name, ns])
    payload = json.dumps(rows).encode()
    parts = gather_bytes(payload, dst, dev, group)
    if parts is None:
        return None
    rows = []
    for p in parts:
        if p:
            rows.extend(json.loads(p.decode()))
    w = AuditWriter(constraints, limit)
    w.set_totals(tot.cpu().tolist(), sweep.actions)
    for r in merge_samples(rows, limit):
        w.add_sample(r[1], (r[7], r[8], r[9]), r[5].encode("latin-1"), r[4], r[6])
    return w
