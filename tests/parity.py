"""Parity harness: run the same driver calls against the HIP engine (gkgpu) and
the CPU oracle (oracle.driver) and compare per-review violation sets.

Comparison unit per review: the multiset of
(constraint kind, constraint name, msg, details JSON, enforcementAction).
The reference iterates constraints and Go-map-backed objects in random order
(SURVEY 8c), so order is not compared.  Reviews the engine routes to the CPU
fallback are excluded from the comparison and counted; reviews it reports as
errors must be errors for the oracle too.
"""
from __future__ import annotations

import collections
import json

from canonical import canonical_row
from gkgpu.client import Client, augmented_review, constraint_path, template_modules
from oracle.driver import OracleDriver, QueryError, TARGET, details_json
from oracle.rego.values import from_json_text


# Templates whose messages %v-print an object, or a set built from an
# object's keys: the reference's byte string depends on Go map order
# (ast/term.go:79-92), so only their rows compare after
# canonicalisation (tests/canonical.py).  Every other row compares byte for
# byte -- e.g. k8srequiredlabels' `missing` set, built from
# parameters.labels[_] in array order
# (demo/agilebank/templates/k8srequiredlabels_template.yaml:39-46), is
# deterministic and must print in that order.
#   K8sPSPHostFilesystem       prints `volume` and input.parameters.allowedHostPaths
#   K8sPSPHostNetworkingPorts  prints input.parameters
#   K8sPSPPrivilegedContainer  prints c.securityContext
#   K8sPSPVolumeTypes          prints {x | volume[x]; x != "name"} (object keys)
# (pkg/webhook/testdata/psp-all-violations/psp-templates/*.yaml)
OBJECT_ORDER_KINDS = frozenset({"K8sPSPHostFilesystem", "K8sPSPHostNetworkingPorts", "K8sPSPPrivilegedContainer",
                                "K8sPSPVolumeTypes"})


def rows_agree(want, got, canonical_kinds=OBJECT_ORDER_KINDS):
    """'exact', 'canonical' (equal only after canonicalising the rows of
    canonical_kinds) or None (a mismatch)."""
    if collections.Counter(want) == collections.Counter(got):
        return "exact"

    def split(rows):
        strict = collections.Counter(r for r in rows if r[0] not in canonical_kinds)
        canon = collections.Counter(canonical_row(r) for r in rows if r[0] in canonical_kinds)
        return strict, canon

    return "canonical" if split(want) == split(got) else None


def oracle_for(templates, constraints, extra_data=()):
    od = OracleDriver()
    for t in templates:
        prefix, mods = template_modules(t)
        od.put_modules(prefix, mods)
    for c in constraints:
        od.put_data(constraint_path(c), json.dumps(c))
    for path, v in extra_data:
        od.put_data(path, json.dumps(v))
    return od


def engine_for(driver, templates, constraints, extra_data=()):
    cl = Client(driver)
    for t in templates:
        cl.add_template(t)
    for c in constraints:
        cl.add_constraint(c)
    for path, v in extra_data:
        driver.put_data(path, v)
    return cl


def oracle_review(od, review):
    """list of result tuples, or the string 'ERROR'."""
    try:
        res = od.query('hooks["%s"].violation' % TARGET, json.dumps({"review": review}))
    except QueryError:
        return "ERROR"
    out = []
    for r in res:
        c = r["constraint"]
        out.append((c.get("kind"), c.get("metadata").get("name"), r["msg"], details_json(r["details"]),
                    r["enforcementAction"]))
    return out


def engine_rows(res, n):
    per = [[] for _ in range(n)]
    for r in res.results:
        per[r.review].append((r.constraint_kind, r.constraint_name, r.msg, r.details_json, r.enforcement_action))
    return per


class Report:
    def __init__(self):
        self.compared = 0
        self.fallback = 0
        self.errors = 0
        self.violations = 0
        self.mismatches = []
        # reviews whose rows agree only after canonicalising printed objects /
        # sets of OBJECT_ORDER_KINDS' rows (Go map order, tests/canonical.py);
        # every other row must be byte-identical
        self.canonical_only = 0

    def __repr__(self):
        return "Report(compared=%d fallback=%d errors=%d violations=%d mismatches=%d canonical_only=%d)" % (
            self.compared, self.fallback, self.errors, self.violations, len(self.mismatches), self.canonical_only)


def compare(od, reviews, eng_res, rep=None):
    rep = rep or Report()
    per = engine_rows(eng_res, len(reviews))
    for i, rv in enumerate(reviews):
        st = eng_res.status[i]
        if st & 2:
            rep.fallback += 1
            continue
        want = oracle_review(od, rv)
        if st & 1:
            rep.errors += 1
            if want != "ERROR":
                rep.mismatches.append((i, "engine error, oracle ok", want, None))
            continue
        if want == "ERROR":
            rep.mismatches.append((i, "oracle error, engine ok", None, per[i]))
            continue
        rep.compared += 1
        rep.violations += len(want)
        how = rows_agree(want, per[i])
        if how == "canonical":
            rep.canonical_only += 1
        elif how is None:
            rep.mismatches.append((i, "diff", want, per[i]))
    return rep


def run_objects(driver, templates, constraints, objs, nss, extra_data=()):
    """Audit discovery mode: Review(AugmentedUnstructured{obj, ns}) for each object."""
    engine_for(driver, templates, constraints, extra_data)
    od = oracle_for(templates, constraints, extra_data)
    res = driver.review_objects(objs, nss)
    reviews = [augmented_review(o, n) for o, n in zip(objs, nss)]
    return compare(od, reviews, res), res
