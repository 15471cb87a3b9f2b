"""HandleViolation (pkg/target/target.go:193-244) against the reference's own
TestHandleViolation cases (target_test.go:273-367) and cases derived from its
code path (tests/golden/gen_handle_violation_cases.py)."""
import json
import os

import pytest

from gkgpu.target import HandleViolationError, handle_violation, resource_identity

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "handle_violation_cases.json")))


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_handle_violation(case):
    if case.get("error"):
        with pytest.raises(HandleViolationError):
            handle_violation(case["review"])
        return
    assert handle_violation(case["review"]) == case["expected"]


def test_reference_cases_present():
    assert sum(1 for c in CASES if c["source"].startswith("pkg/target/target_test.go")) == 3


def test_resource_identity_getters():
    assert resource_identity({"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "a", "namespace": "b"}}) == \
        ("v1", "Pod", "a", "b")
    assert resource_identity({"kind": "Pod", "metadata": {"name": 7}}) == ("", "Pod", "", "")
