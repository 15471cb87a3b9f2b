"""Replay the reference's match-library KATs (tests/golden/match_kats.jsonl,
recorded from pkg/target/regolib/*_test.rego by gen_match_kats.py) through the
engine's full match stage: each function-level vector becomes a (constraint,
review, namespace cache) triple evaluated with a deny-all template, so a
violation appears iff matching_constraints holds (plus the autoreject result
for autoreject_review vectors, target_template_source.go:12-25).

Expected rows come from the oracle driver on the same triple (the oracle's
match library is pinned by these very vectors, test_oracle_match_kats.py);
`direct` marks vectors whose function alone decides the match (every other
match criterion defaults to true), where the KAT's own result is the
expectation too."""
from __future__ import annotations

import json
import os

from parity import oracle_for
from gkgpu import workloads as W
from gkgpu.client import TARGET

HERE = os.path.dirname(os.path.abspath(__file__))
UNDEF = object()
DENY_ALL = W._tmpl("K8sDenyAll", 'package k8sdenyall\n\nviolation[{"msg": msg}] {\n\tmsg := "denied"\n}\n')
MATCH_FNS = ("matches_label_selector", "any_labelselector_match", "any_kind_selector_matches", "matches_scope",
             "matches_namespaces", "does_not_match_excludednamespaces", "matches_nsselector", "autoreject_review")


def plain(x):
    """codec form -> JSON-able value (object key order kept), UNDEF for #u"""
    if isinstance(x, list):
        return [plain(e) for e in x]
    if isinstance(x, dict):
        if "#u" in x:
            return UNDEF
        if "#n" in x:
            return json.loads(x["#n"])
        if "#o" in x:
            return {k: plain(v) for k, v in x["#o"]}
        if "#s" in x:
            return [plain(e) for e in x["#s"]]
    return x


def cases():
    out = []
    for i, line in enumerate(open(os.path.join(HERE, "golden", "match_kats.jsonl"))):
        v = json.loads(line)
        fn = v["fn"]
        if fn not in MATCH_FNS:
            continue
        args = [plain(a) for a in v["args"]]
        inp = plain(v["input"])
        review = inp.get("review", UNDEF) if isinstance(inp, dict) else UNDEF
        ext = plain(v["external"])
        cache = {}
        if isinstance(ext, dict):
            cache = ((ext.get("cluster") or {}).get("v1") or {}).get("Namespace") or {}
        constraints = []
        direct = True
        if fn == "autoreject_review":
            root = plain(v["constraints"])
            for kind, named in (root.items() if isinstance(root, dict) else []):
                for name, c in named.items():
                    constraints.append((kind, name, c))
        else:
            if fn == "matches_label_selector":
                match = {"labelSelector": args[0]}
                review = {"kind": {"group": "", "version": "v1", "kind": "Thing"},
                          "object": {"metadata": {"labels": args[1]}}}
            elif fn == "any_labelselector_match":
                match = {"labelSelector": args[0]}
            else:
                match = args[0]
            constraints.append(("K8sDenyAll", "c", {"apiVersion": "constraints.gatekeeper.sh/v1beta1",
                                                    "kind": "K8sDenyAll", "metadata": {"name": "c"},
                                                    "spec": {"match": match}}))
        result = plain(v["result"])
        out.append({"id": "%s#%d" % (v["test"].split(":")[1], i), "fn": fn, "constraints": constraints,
                    "cache": cache, "review": review, "kat": result})
    return out


def extra_data(case):
    data = [("/constraints/%s/cluster/constraints.gatekeeper.sh/%s/%s" % (TARGET, k, n), c)
            for k, n, c in case["constraints"]]
    data += [("/external/%s/cluster/v1/Namespace/%s" % (TARGET, n), o) for n, o in case["cache"].items()]
    return data


def query_input(case):
    return {} if case["review"] is UNDEF else {"review": case["review"]}


def expected(case):
    """oracle rows for the triple: sorted [(msg, details JSON, enforcementAction)] or 'ERROR'"""
    from oracle.driver import QueryError, details_json
    od = oracle_for([DENY_ALL], [], extra_data(case))
    try:
        res = od.query('hooks["%s"].violation' % TARGET, json.dumps(query_input(case)))
    except QueryError:
        return "ERROR"
    return sorted((r["msg"], details_json(r["details"]), r["enforcementAction"]) for r in res)


def engine_for(drv, case):
    from gkgpu.client import Client
    cl = Client(drv)
    cl.add_template(DENY_ALL)
    for path, v in extra_data(case):
        drv.put_data(path, v)
    return cl
