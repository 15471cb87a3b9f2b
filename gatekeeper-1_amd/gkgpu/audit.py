"""Audit results writer: the consumer of the violation set.

Restates pkg/audit/manager.go for the results of one sweep:
  * addAuditResponsesToUpdateLists (:462-508) -- per-constraint totals, the
    first `limit` results per constraint in evaluation order, per-action totals
    keyed by the raw enforcementAction string (deny/dryrun/unrecognized
    pre-zeroed, :190-193);
  * updateConstraintStatus (:555-631) -- status.violations[] entries
    {kind, name, namespace (omitempty), message, enforcementAction}, messages
    over msgSize (256) bytes cut by truncateString (:623-631), plus
    totalViolations; an empty list removes status.violations.
The resource fields come from HandleViolation (pkg/target/target.go:193-244):
the review's object (else oldObject) with kind = review.kind.kind.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

MSG_SIZE = 256                      # manager.go:41
DEFAULT_LIMIT = 20                  # manager.go:43 (--constraint-violations-limit)
KNOWN_ACTIONS = ("deny", "dryrun", "unrecognized")  # pkg/util/enforcement_action.go:11-17


def truncate_bytes(head: bytes, total_len: int, size: int = MSG_SIZE) -> str:
    """truncateString (manager.go:623-631) of a message known by its first
    bytes `head` (at least min(total_len, size) of them) and its byte length;
    the status is JSON, so a cut inside a UTF-8 sequence marshals as U+FFFD."""
    if total_len <= size:
        return head[:total_len].decode("utf-8", "surrogateescape")
    cut = size - 3 if size > 3 else size
    return (head[:cut] + b"...").decode("utf-8", "replace")


def truncate_string(msg: str, size: int = MSG_SIZE) -> str:
    """truncateString (manager.go:623-631) on the message's bytes"""
    b = msg.encode("utf-8", "surrogateescape")
    if len(b) <= size:
        return msg
    return truncate_bytes(b, len(b), size)


class AuditWriter:
    """Accumulates one audit sweep's results (in evaluation order) per constraint."""

    def __init__(self, constraints: Sequence[Tuple[str, str]], limit: int = DEFAULT_LIMIT):
        self.constraints = list(constraints)        # engine constraint index -> (kind, name)
        self.limit = limit
        self.totals: Dict[int, int] = {}
        self.samples: Dict[int, List[dict]] = {}
        self.per_action: Dict[str, int] = {a: 0 for a in KNOWN_ACTIONS}

    def add(self, constraint: int, resource: Tuple[str, str, str], msg: str, enforcement_action: str):
        """one types.Result: resource = (kind, name, namespace)"""
        self.totals[constraint] = self.totals.get(constraint, 0) + 1
        lst = self.samples.setdefault(constraint, [])
        if len(lst) < self.limit:
            kind, name, ns = resource
            lst.append({"kind": kind, "name": name, "namespace": ns, "message": msg,
                        "enforcementAction": enforcement_action})
        self.per_action[enforcement_action] = self.per_action.get(enforcement_action, 0) + 1

    def add_sample(self, constraint: int, resource: Tuple[str, str, str], head: bytes, msg_len: int,
                   enforcement_action: str):
        """one sampled result whose message is known by its first bytes (the
        engine's device sample, gk_results_sample_get); totals come separately"""
        lst = self.samples.setdefault(constraint, [])
        if len(lst) < self.limit:
            kind, name, ns = resource
            lst.append({"kind": kind, "name": name, "namespace": ns, "final": truncate_bytes(head, msg_len),
                        "enforcementAction": enforcement_action})

    def set_totals(self, totals: Sequence[int], actions: Sequence[str]):
        """per-constraint totals of a sweep and the per-action totals they imply
        (every result of a constraint carries its enforcementAction)"""
        self.totals = {c: int(n) for c, n in enumerate(totals) if n}
        self.per_action = {a: 0 for a in KNOWN_ACTIONS}
        for c, n in enumerate(totals):
            if n:
                self.per_action[actions[c]] = self.per_action.get(actions[c], 0) + int(n)

    @staticmethod
    def from_sweep(constraints, sweep, resource_of_review, limit: int = DEFAULT_LIMIT, fallback=None) -> "AuditWriter":
        """status writer of one engine sweep (Batch.eval_audit);
        resource_of_review(i) -> (kind, name, namespace).  Reviews the engine
        flagged (sweep.flagged: error / CPU fallback) are answered by
        `fallback(i)` -> [(constraint index, msg, enforcementAction)] in the
        reference's per-review order, e.g. the embedded CPU OPA driver, and
        merged in at their position in evaluation order; without a fallback a
        sweep with flagged reviews raises (its status would silently miss
        them).  A review whose Query errors returns [] (manager.go:376-381
        skips it)."""
        totals, rows = flagged_rows(sweep, fallback, 0)
        w = AuditWriter(constraints, limit)
        w.set_totals(totals, sweep.actions)
        for s in sweep.samples:
            rows.append((s.review, 0 if s.rule == 0xffff else 1, s.seq, s.constraint, s.msg, s.msg_len, s.enforcement_action))
        rows.sort(key=lambda r: (r[3], r[0], r[1], r[2]))
        for rv, _ar, _seq, c, head, ml, ea in rows:
            w.add_sample(c, resource_of_review(rv), head, ml, ea)
        return w

    def add_results(self, results, resources: Sequence[Tuple[str, str, str]]):
        """engine or oracle results, already in evaluation order (review, then
        the per-review result order), each with .review/.constraint/.msg/
        .enforcement_action; resources[review] = (kind, name, namespace)"""
        for r in results:
            self.add(r.constraint, resources[r.review], r.msg, r.enforcement_action)

    def status(self, constraint: int) -> dict:
        """the constraint's status fields written by updateConstraintStatus"""
        out = {"totalViolations": self.totals.get(constraint, 0)}
        vs = []
        for ar in self.samples.get(constraint, [])[: self.limit]:
            v = {"kind": ar["kind"], "name": ar["name"]}
            if ar["namespace"]:
                v["namespace"] = ar["namespace"]
            v["message"] = ar["final"] if "final" in ar else truncate_string(ar["message"])
            v["enforcementAction"] = ar["enforcementAction"]
            vs.append(v)
        if vs:
            out["violations"] = vs
        return out

    def statuses(self) -> Dict[Tuple[str, str], dict]:
        return {self.constraints[i]: self.status(i) for i in range(len(self.constraints))}

    @staticmethod
    def merge(writers: Sequence["AuditWriter"]) -> "AuditWriter":
        """Rank-order merge of per-shard writers (contiguous resource shards,
        rank r holding the r-th range): totals add, samples concatenate in rank
        order up to the limit -- the single-process sweep's result."""
        w0 = writers[0]
        m = AuditWriter(w0.constraints, w0.limit)
        for w in writers:
            for c, n in w.totals.items():
                m.totals[c] = m.totals.get(c, 0) + n
            for c, lst in w.samples.items():
                dst = m.samples.setdefault(c, [])
                dst.extend(lst[: max(0, m.limit - len(dst))])
            for a, n in w.per_action.items():
                m.per_action[a] = m.per_action.get(a, 0) + n
        return m


class FlaggedReviews(RuntimeError):
    """an engine sweep flagged reviews (error / CPU fallback) and no fallback
    evaluator was given to answer them"""


def flagged_rows(sweep, fallback, review_base: int):
    """(totals including the flagged reviews' results, sample rows of those
    results) -- rows (global review, autoreject last key 1, order, constraint,
    message bytes, message length, enforcementAction)"""
    totals = [int(x) for x in sweep.totals]
    rows = []
    flagged = list(getattr(sweep, "flagged", []) or [])
    if not flagged:
        return totals, rows
    if fallback is None:
        raise FlaggedReviews("%d reviews flagged error/fallback need the CPU driver (pass fallback=)" % len(flagged))
    for rv in flagged:
        for j, (c, msg, ea) in enumerate(fallback(rv)):
            if c >= len(totals):
                totals.extend([0] * (c + 1 - len(totals)))
            totals[c] += 1
            b = msg.encode("utf-8", "surrogateescape")
            rows.append((int(review_base) + rv, 1, j, c, b[:MSG_SIZE], len(b), ea))
    return totals, rows


def resource_of(review_or_object: dict, is_review: bool = False) -> Tuple[str, str, str]:
    """(kind, name, namespace) of HandleViolation's Resource (target.go:193-244)."""
    if is_review:
        kind = (review_or_object.get("kind") or {}).get("kind", "")
        obj = review_or_object.get("object") or review_or_object.get("oldObject") or {}
    else:
        obj = review_or_object
        kind = obj.get("kind", "")
    md = obj.get("metadata") or {}
    return kind, md.get("name", "") or "", md.get("namespace", "") or ""
