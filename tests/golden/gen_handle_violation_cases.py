"""Write tests/golden/handle_violation_cases.json: TestHandleViolation
(pkg/target/target_test.go:273-367) transliterated as data -- review JSON in,
expected Result.Resource object (or an expected error) out -- plus cases
derived from HandleViolation's code path (pkg/target/target.go:165-244) that
the reference test does not exercise: the oldObject fallback, a null object
treated as missing (nestedMap, :180-191), a non-string kind field (getString,
:165-178), a review without object or oldObject, and a 3-part apiVersion.
Those derived cases are pinned by the code reading only ("source": "derived")."""
import json
import os

REF = "pkg/target/target_test.go:273-367"
DER = "derived: pkg/target/target.go:165-244"

CASES = [
    {"name": "Valid Review", "source": REF,
     "review": {"kind": {"group": "myGroup", "version": "v1", "kind": "MyKind"}, "name": "somename",
                "operation": "CREATE", "object": {"metadata": {"name": "somename"}, "spec": {"value": "yep"}}},
     "expected": {"apiVersion": "myGroup/v1", "kind": "MyKind", "metadata": {"name": "somename"},
                  "spec": {"value": "yep"}}},
    {"name": "Valid Review (No Group)", "source": REF,
     "review": {"kind": {"group": "", "version": "v1", "kind": "MyKind"}, "name": "somename",
                "operation": "CREATE", "object": {"metadata": {"name": "somename"}, "spec": {"value": "yep"}}},
     "expected": {"apiVersion": "v1", "kind": "MyKind", "metadata": {"name": "somename"}, "spec": {"value": "yep"}}},
    {"name": "No Review", "source": REF, "review": ["list is wrong"], "error": True},
    {"name": "oldObject when object is missing", "source": DER,
     "review": {"kind": {"group": "apps", "version": "v1", "kind": "Deployment"},
                "oldObject": {"metadata": {"name": "old", "namespace": "ns1"}}},
     "expected": {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "old", "namespace": "ns1"}}},
    {"name": "null object is missing", "source": DER,
     "review": {"kind": {"group": "", "version": "v1", "kind": "Pod"}, "object": None,
                "oldObject": {"metadata": {"name": "p"}, "kind": "Other", "apiVersion": "x/y"}},
     "expected": {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "p"}}},
    {"name": "object wins over oldObject", "source": DER,
     "review": {"kind": {"group": "", "version": "v1", "kind": "Pod"}, "object": {"metadata": {"name": "new"}},
                "oldObject": {"metadata": {"name": "old"}}},
     "expected": {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": "new"}}},
    {"name": "non-string kind field", "source": DER,
     "review": {"kind": {"group": "", "version": 1, "kind": "Pod"}, "object": {}}, "error": True},
    {"name": "missing group", "source": DER,
     "review": {"kind": {"version": "v1", "kind": "Pod"}, "object": {}}, "error": True},
    {"name": "no object or oldObject", "source": DER,
     "review": {"kind": {"group": "", "version": "v1", "kind": "Pod"}}, "error": True},
    {"name": "object is not a map", "source": DER,
     "review": {"kind": {"group": "", "version": "v1", "kind": "Pod"}, "object": "str"}, "error": True},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "handle_violation_cases.json")
    with open(out, "w") as f:
        json.dump(CASES, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", out, len(CASES))
