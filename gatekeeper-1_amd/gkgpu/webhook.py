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

* ``handle_requests``  — Handle's steps ahead of the engine for raw
  AdmissionRequests: the Gatekeeper service-account bypass (policy.go:147-149,
  304-306), DELETE reviewing oldObject (:151-166), the webhook process
  excluder (:192-196, 425-427) and the Namespace fetch of reviewRequest
  (:372-383: the cached client first, the API reader on NotFound, any other
  error fails the request with 500), then one ``handle_batch`` launch for the
  requests that reach the engine.

Validation of Gatekeeper's own resources (validateGatekeeperResources,
:168-179: ConstraintTemplate / constraint admission) is the control plane's and
out of scope.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

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


# -- Handle's steps ahead of the engine (policy.go:142-223, 363-400) --------------

class NotFound(Exception):
    """k8serrors.IsNotFound for a Namespace Get."""


class NamespaceFetcher:
    """reviewRequest's Namespace lookup (policy.go:372-383): the cached client
    (h.client.Get) first; only on NotFound the API reader (h.reader.Get, which
    bypasses the cache); any other error, or the reader's error, fails the
    request.  `cache_get(name)` / `reader_get(name)` return the Namespace
    object or raise (NotFound for a missing one)."""

    def __init__(self, cache_get: Callable[[str], dict], reader_get: Callable[[str], dict]):
        self.cache_get = cache_get
        self.reader_get = reader_get

    def get(self, name: str) -> dict:
        try:
            return self.cache_get(name)
        except NotFound:
            return self.reader_get(name)


def gk_service_account() -> str:
    """serviceaccount (policy.go:67, 77): system:serviceaccount:<POD_NAMESPACE,
    default gatekeeper-system (pkg/util/pod_info.go:15-21)>:gatekeeper-admin"""
    return "system:serviceaccount:%s:gatekeeper-admin" % os.environ.get("POD_NAMESPACE", "gatekeeper-system")


def handle_requests(driver, requests: Sequence[dict], fetcher: NamespaceFetcher) -> List[Response]:
    """Handle (policy.go:142-223) for a micro-batch of AdmissionRequests (dicts
    in admission/v1beta1 JSON form): the host steps per request, then one
    engine launch for every request that reaches reviewRequest's Review."""
    out: List[Optional[Response]] = [None] * len(requests)
    inputs, where = [], []
    for i, req in enumerate(requests):
        user = (req.get("userInfo") or {}).get("username", "")
        if user == gk_service_account():
            out[i] = Response(True, ALLOWED, "Gatekeeper does not self-manage")
            continue
        if req.get("operation") == "DELETE":
            if req.get("oldObject") is None:
                out[i] = Response(False, ERROR, "For admission webhooks registered for DELETE operations, "
                                                 "please use Kubernetes v1.15.0+.")
                continue
            req = dict(req)
            req["object"] = req["oldObject"]
        if driver.is_namespace_excluded("webhook", req.get("namespace", "") or ""):
            out[i] = Response(True, ALLOWED, "Namespace is set to be ignored by Gatekeeper config")
            continue
        kind = req.get("kind") or {}
        ns_name = "" if (kind.get("kind") == "Namespace" and kind.get("group", "") == "") else (req.get("namespace") or "")
        ns = None
        if ns_name:
            try:
                ns = fetcher.get(ns_name)
            except Exception as err:  # reviewRequest's error: Handle answers 500 with its text
                out[i] = Response(False, ERROR, str(err))
                continue
        inputs.append(review_input(req, ns))
        where.append(i)
    if inputs:
        for i, r in zip(where, handle_batch(driver, inputs)):
            out[i] = r
    return out
