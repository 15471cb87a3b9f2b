"""Audit results writer (pkg/audit/manager.go:462-508, 555-631) on the host."""
from gkgpu.audit import AuditWriter, truncate_string, resource_of


class R:
    def __init__(self, review, constraint, msg, ea="deny"):
        self.review, self.constraint, self.msg, self.enforcement_action = review, constraint, msg, ea


def test_truncate_string_matches_go():
    assert truncate_string("a" * 256) == "a" * 256
    assert truncate_string("a" * 257) == "a" * 253 + "..."
    assert len(truncate_string("x" * 1000).encode()) == 256
    # a cut inside a multi-byte rune marshals as U+FFFD (encoding/json)
    s = "a" * 252 + "é" + "b" * 10
    assert truncate_string(s) == "a" * 252 + "�..."


def test_limit_totals_and_actions():
    w = AuditWriter([("K8sA", "a"), ("K8sB", "b")], limit=3)
    res = [R(i, i % 2, "m%d" % i, "dryrun" if i % 5 == 0 else "deny") for i in range(10)] + [R(11, 1, "x", "warn")]
    resources = [("Pod", "p%d" % i, "ns" if i % 3 else "") for i in range(12)]
    w.add_results(res, resources)
    assert w.totals == {0: 5, 1: 6}
    assert w.per_action == {"deny": 8, "dryrun": 2, "unrecognized": 0, "warn": 1}
    st = w.status(0)
    assert st["totalViolations"] == 5
    assert [v["message"] for v in st["violations"]] == ["m0", "m2", "m4"]
    assert "namespace" not in st["violations"][0] and st["violations"][1]["namespace"] == "ns"
    assert w.status(1)["violations"][0] == {"kind": "Pod", "name": "p1", "namespace": "ns", "message": "m1",
                                            "enforcementAction": "deny"}


def test_empty_status_has_no_violations_field():
    w = AuditWriter([("K8sA", "a")])
    assert w.status(0) == {"totalViolations": 0}


def test_rank_order_merge_equals_single_sweep():
    res = [R(i, i % 3, "m%d" % i) for i in range(100)]
    resources = [("Pod", "p%d" % i, "default") for i in range(100)]
    whole = AuditWriter([("K", "a"), ("K", "b"), ("K", "c")], limit=20)
    whole.add_results(res, resources)
    parts = []
    for lo, hi in ((0, 33), (33, 66), (66, 100)):
        w = AuditWriter(whole.constraints, limit=20)
        w.add_results([r for r in res if lo <= r.review < hi], resources)
        parts.append(w)
    m = AuditWriter.merge(parts)
    assert m.statuses() == whole.statuses()
    assert m.per_action == whole.per_action


def test_resource_of_review_and_object():
    rv = {"kind": {"group": "", "version": "v1", "kind": "Pod"}, "object": None,
          "oldObject": {"metadata": {"name": "old", "namespace": "x"}}}
    assert resource_of(rv, is_review=True) == ("Pod", "old", "x")
    assert resource_of({"kind": "Namespace", "metadata": {"name": "n"}}) == ("Namespace", "n", "")
