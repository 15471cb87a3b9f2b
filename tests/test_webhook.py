"""Admission-webhook micro-batch path (pkg/webhook/policy.go) on the host side:
deny-message assembly, review shape, and the config-5 workload against the oracle."""
import json

from gkgpu import workloads as W
from gkgpu.webhook import DENIED, ALLOWED, ERROR, FALLBACK, deny_messages, namespace_object, respond, review_input

from parity import oracle_for, oracle_review


class R:
    def __init__(self, name, ea, msg="test"):
        self.constraint_name, self.enforcement_action, self.msg = name, ea, msg


def test_get_deny_messages_counts():
    """TestGetDenyMessages (pkg/webhook/policy_test.go:550-643)."""
    dry, deny, rnd = R("ph", "dryrun"), R("ph", "deny"), R("ph", "random")
    cases = [([dry], 0), ([deny], 1), ([dry, deny], 1), ([deny, deny], 2), ([dry, dry], 0), ([rnd], 0)]
    for res, n in cases:
        assert len(deny_messages(res)) == n
    assert deny_messages([deny]) == ["[denied by ph] test"]


def test_respond_codes():
    assert respond(0, []).code == ALLOWED and respond(0, []).allowed
    r = respond(0, [R("a", "deny", "m1"), R("b", "dryrun", "m2"), R("c", "deny", "m3")])
    assert (r.allowed, r.code, r.message) == (False, DENIED, "[denied by a] m1\n[denied by c] m3")
    assert respond(1, []).code == ERROR
    assert respond(2, []).code == FALLBACK


def test_review_input_shape():
    """AugmentedReview -> gkReview (target.go:42-60, 95-100); Namespace-kind
    coercion (policy.go:366-371)."""
    req = W.admission_request(7, __import__("random").Random(1))
    rv = review_input(req, namespace_object(req["namespace"]))["review"]
    keys = list(rv)
    assert keys[:3] == ["uid", "kind", "resource"] and keys[-1] == "_unstable"
    assert rv["_unstable"]["namespace"]["metadata"] == {"name": "res-namespace-7", "creationTimestamp": None}
    assert rv["object"]["metadata"]["resourceVersion"] == "2" and rv["oldObject"]["metadata"]["resourceVersion"] == "1"
    assert rv["operation"] == "UPDATE" and rv["dryRun"] is False and rv["options"] is None
    nsreq = {"kind": {"group": "", "version": "v1", "kind": "Namespace"}, "namespace": "x", "operation": "CREATE"}
    nrv = review_input(nsreq, None)["review"]
    assert "namespace" not in nrv and nrv["_unstable"] == {}


def test_config5_constraint_load_names():
    """generateConstraints (policy_benchmark_test.go:176-186): first round keeps
    the names, later copies get fresh random names."""
    ts, cs = W.config5(12)
    assert len(ts) == 5 and len(cs) == 12
    names = [c["metadata"]["name"] for c in cs]
    assert names[:5] == [c["metadata"]["name"] for c in W.PSP_CONSTRAINTS]
    assert len(set(names)) == 12 and all(len(n) == 10 for n in names[5:])
    assert [c["kind"] for c in cs] == [W.PSP_CONSTRAINTS[i % 5]["kind"] for i in range(12)]


def test_config5_oracle_all_violating():
    """'psp: 100% violations' (policy_benchmark_test.go:253-262): every request
    is denied; messages follow the PSP templates."""
    ts, cs = W.config5(5)
    od = oracle_for(ts, cs)
    ins = W.gen_admission_inputs(10)
    for i, s in enumerate(ins):
        res = oracle_review(od, json.loads(s)["review"])
        assert res != "ERROR" and len(res) >= 1
        assert all(r[4] == "deny" for r in res)
    r1 = oracle_review(od, json.loads(ins[1])["review"])
    assert [r[2] for r in r1] == ["Sharing the host namespace is not allowed: res-name-1"]
