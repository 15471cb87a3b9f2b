"""Diagnostic: the from-cache audit's rows against the oracle's, printing the
rows each side lacks (tests/test_audit_cache.py's namespace-selector setup)."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "gatekeeper-1_amd")]
import test_audit_cache as T  # noqa: E402
from oracle.driver import details_json  # noqa: E402

d, cl, od, cs, items, synced = T._nssel_setup(1500, 42, False)
order = sorted(p for p, _ in items)
res = cl.audit()
got = collections.Counter()
for r in res.results:
    seg = order[r.review].split("/")
    got[(seg[-1], r.constraint_name, r.msg)] += 1
want = collections.Counter()
for r in T._oracle_rows(od):
    want[(r["review"].get("name"), r["constraint"].get("metadata").get("name"), r["msg"])] += 1
miss, extra = want - got, got - want
print("flagged reviews", sum(1 for s in res.status if s))
print("rows got", sum(got.values()), "want", sum(want.values()), "missing", sum(miss.values()), "extra", sum(extra.values()))
idx = {pth.split("/")[-1]: i for i, pth in enumerate(order)}
for k, n in list(miss.items())[:40]:
    print("MISSING", n, idx.get(k[0]), k)
for k, n in list(extra.items())[:20]:
    print("EXTRA", n, k)
