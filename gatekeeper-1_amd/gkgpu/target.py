"""K8s target handler steps that run on the Client side of the driver.

HandleViolation (pkg/target/target.go:193-244): every Result of a Review gets
Result.Resource = the review's object (else oldObject) with apiVersion and kind
overwritten from review.kind; an error fails the whole Review for the target
(client.go:786-791).  The batch audit path gets the same identity from the
engine (gk_batch_resource) without materialising objects.
"""
from __future__ import annotations

import copy
from typing import Tuple


class HandleViolationError(ValueError):
    pass


def _get_string(review: dict, k: str) -> str:
    """getString (target.go:165-178): review["kind"][k] must exist and be a string."""
    kind = review.get("kind")
    if not isinstance(kind, dict):
        if kind is None:
            raise HandleViolationError("review[kind][%s] does not exist" % k)
        raise HandleViolationError(".kind accessor error: %r is of the type %s, expected map[string]interface{}"
                                   % (kind, type(kind).__name__))
    if k not in kind:
        raise HandleViolationError("review[kind][%s] does not exist" % k)
    v = kind[k]
    if not isinstance(v, str):
        raise HandleViolationError("review[kind][%s] is not a string: %r" % (k, v))
    return v


def _nested_map(review: dict, field: str):
    """nestedMap (target.go:180-191): (map, found); a null value is missing,
    any other non-map value is an error"""
    if field not in review or review[field] is None:
        return None, False
    v = review[field]
    if not isinstance(v, dict):
        raise HandleViolationError("%s accessor error: %r is of the type %s, expected map[string]interface{}"
                                   % (field, v, type(v).__name__))
    return v, True


def handle_violation(review) -> dict:
    """Result.Resource for a result of `review` (target.go:193-244)."""
    if not isinstance(review, dict):
        raise HandleViolationError("could not cast review as map[string]: %r" % (review,))
    group = _get_string(review, "group")
    version = _get_string(review, "version")
    kind = _get_string(review, "kind")
    api_version = version if group == "" else "%s/%s" % (group, version)
    obj, found = _nested_map(review, "object")
    if not found:
        obj, found = _nested_map(review, "oldObject")
        if not found:
            raise HandleViolationError("no object or oldObject returned in review")
    res = copy.deepcopy(obj)
    res["apiVersion"] = api_version
    res["kind"] = kind
    return res


def resource_identity(resource: dict) -> Tuple[str, str, str, str]:
    """(apiVersion, kind, name, namespace) as unstructured's getters read them
    (GetName/GetNamespace return "" for missing or non-string values)."""
    md = resource.get("metadata") if isinstance(resource.get("metadata"), dict) else {}
    s = lambda v: v if isinstance(v, str) else ""  # noqa: E731
    return s(resource.get("apiVersion")), s(resource.get("kind")), s(md.get("name")), s(md.get("namespace"))
