"""Write tests/golden/integration_cases.json: the 23 cases of
pkg/target/target_integration_test.go:141-363 (TestConstraintEnforcement),
transliterated as data (object group/kind/labels, namespace name/labels,
constraint match builders, expected allowed).  Each case is reviewed three ways
by the reference test (:405-461): AdmissionRequest.object, .oldObject, and
AugmentedUnstructured; the expected outcome is the same for all three.
"""
import json
import os

OBJ = {"group": "some", "kind": "Thing"}


def obj(labels=None):
    return dict(OBJ, labels=labels)


def ns(name, labels=None):
    return {"name": name, "labels": labels}


def kinds(groups, ks):
    return {"kinds": [{"apiGroups": groups, "kinds": ks}]}


def every(scope=None, kinds_groups=("some",), nsname="my-ns", lsel=("obj", "label"), nssel=("ns", "label")):
    m = {}
    m.update(kinds(list(kinds_groups), ["Thing"]))
    if scope:
        m["scope"] = scope
    m["namespaces"] = [nsname]
    m["labelSelector"] = {"matchLabels": {lsel[0]: lsel[1]}}
    m["namespaceSelector"] = {"matchLabels": {nssel[0]: nssel[1]}}
    return m


L = {"obj": "label"}
NSL = {"ns": "label"}
CASES = [
    ("match deny all", obj(), ns("my-ns"), None, False),
    ("match namespace", obj(), ns("my-ns"), {"namespaces": ["my-ns"]}, False),
    ("no match namespace", obj(), ns("my-ns"), {"namespaces": ["not-my-ns"]}, True),
    ("match excludedNamespaces", obj(), ns("my-ns"), {"excludedNamespaces": ["my-ns"]}, True),
    ("no match excludedNamespaces", obj(), ns("my-ns"), {"excludedNamespaces": ["not-my-ns"]}, False),
    ("match labelselector", obj({"a": "label"}), ns("my-ns"), {"labelSelector": {"matchLabels": {"a": "label"}}}, False),
    ("no match labelselector", obj({"a": "label"}), ns("my-ns"), {"labelSelector": {"matchLabels": {"different": "label"}}}, True),
    ("match nsselector", obj(), ns("my-ns", {"a": "label"}), {"namespaceSelector": {"matchLabels": {"a": "label"}}}, False),
    ("no match nsselector", obj(), ns("my-ns", {"a": "label"}), {"namespaceSelector": {"matchLabels": {"different": "label"}}}, True),
    ("match kinds", obj(), ns("my-ns"), kinds(["some"], ["Thing"]), False),
    ("no match kinds", obj(), ns("my-ns"), kinds(["different"], ["Thing"]), True),
    ("match everything", obj(L), ns("my-ns", NSL), every(), False),
    ("match everything with scope as wildcard", obj(L), ns("my-ns", NSL), every("*"), False),
    ("match everything with scope as namespaced", obj(L), ns("my-ns", NSL), every("Namespaced"), False),
    ("match everything with scope as cluster", obj(L), ns("my-ns", NSL), every("Cluster"), True),
    ("match everything but kind", obj(L), ns("my-ns", NSL), every(kinds_groups=("different",)), True),
    ("match everything but namespace", obj(L), ns("my-ns", NSL), every(nsname="different-ns"), True),
    ("match everything but labelselector", obj(L), ns("my-ns", NSL), every(lsel=("obj", "different-label")), True),
    ("match everything but nsselector", obj(L), ns("my-ns", NSL), every(nssel=("ns", "different-label")), True),
    ("match everything cluster scoped", obj(L), None, every(), False),
    ("match everything cluster scoped wildcard as scope", obj(L), None, every("*"), False),
    ("do not match everything cluster scoped namespaced as scope", obj(L), None, every("Namespaced"), True),
    ("match everything cluster scoped with cluster as scope", obj(L), None, every("Cluster"), False),
]


def main():
    out = []
    for name, o, n, m, allowed in CASES:
        out.append({"name": name, "object": o, "namespace": n, "match": m, "allowed": allowed})
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "integration_cases.json")
    with open(p, "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    print(len(out), "cases ->", p)


if __name__ == "__main__":
    main()
