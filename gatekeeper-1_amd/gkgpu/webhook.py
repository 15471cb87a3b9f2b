"""Admission-webhook path on the batch engine (BASELINE config 5).

Mirrors pkg/webhook/policy.go for the part that reaches the policy engine:

* ``review_input``     — reviewRequest (policy.go:363-400): the Namespace-kind
  coercion, then ``AugmentedReview{AdmissionRequest, Namespace}`` which the
  target turns into ``gkReview`` with ``_unstable.namespace``
  (pkg/target/target.go:42-60, 95-100);
* ``deny_messages``    — getDenyMessages (policy.go:225-291): only results with
  enforcementAction ``deny`` produce ``[denied by <constraint>] <msg>``;
* ``handle_batch``     — Handle (policy.go:142-223) for a micro-batch: one
  ``gk_query_batch`` launch evaluates up to 256 requests; each request gets the
  response Handle would build (allowed / 403 with the joined deny messages /
  500 on a Query error).  Requests the engine flags for fallback are returned
  as such: the caller re-runs them on the CPU driver.

The service-account bypass, DELETE handling of oldObject and the Gatekeeper
self-validation steps of Handle run before the engine and are out of scope.
"""
from __future__ import annotations

import json
from dataclasses import dataclass
from typing import List, Optional, Sequence

from .driver import GK_REVIEW_ERROR, GK_REVIEW_FALLBACK, TARGET

VIOLATION_PATH = 'hooks["%s"].violation' % TARGET

# Handle's response codes (policy.go:196-222)
ALLOWED = 200
DENIED = 403      # http.StatusForbidden
ERROR = 500       # http.StatusInternalServerError
FALLBACK = -1     # engine asks for the CPU driver


def namespace_object(name: str) -> dict:
    """corev1.Namespace{ObjectMeta{Name}} marshalled by encoding/json: what the
    webhook's namespace Get returns in policy_benchmark_test.go:56-65."""
    return {"metadata": {"name": name, "creationTimestamp": None}, "spec": {}, "status": {}}


def review_input(request: dict, ns: Optional[dict]) -> dict:
    """{"review": gkReview} for Review(&AugmentedReview{req, ns}) (policy.go:363-387).

    A Namespace-kind request in the core group is reviewed with namespace ""
    (policy.go:366-371); ns is the Namespace object the webhook fetched, or
    None when the request has no namespace (``_unstable: {}``: the
    ``Namespace`` pointer is omitempty, target.go:57-60)."""
    req = dict(request)
    kind = req.get("kind") or {}
    if kind.get("kind") == "Namespace" and kind.get("group", "") == "":
        req.pop("namespace", None)
    unstable = {} if ns is None else {"namespace": ns}
    req["_unstable"] = unstable
    return {"review": req}


def deny_messages(results) -> List[str]:
    """getDenyMessages (policy.go:225-291): one message per result whose
    enforcementAction is exactly "deny", in result order."""
    return ["[denied by %s] %s" % (r.constraint_name, r.msg) for r in results if r.enforcement_action == "deny"]


@dataclass
class Response:
    allowed: bool
    code: int
    message: str


def respond(status: int, results) -> Response:
    """Handle's decision for one request from its engine status and results."""
    if status & GK_REVIEW_FALLBACK:
        return Response(False, FALLBACK, "")
    if status & GK_REVIEW_ERROR:
        return Response(False, ERROR, "error executing query")
    msgs = deny_messages(results)
    if msgs:
        return Response(False, DENIED, "\n".join(msgs))
    return Response(True, ALLOWED, "")


def handle_batch(driver, inputs: Sequence) -> List[Response]:
    """One micro-batch: inputs are review_input() dicts or their JSON text."""
    res = driver.query_batch([x if isinstance(x, str) else json.dumps(x) for x in inputs])
    per = [[] for _ in range(len(inputs))]
    for r in res.results:
        per[r.review].append(r)
    return [respond(res.status[i], per[i]) for i in range(len(inputs))]
