"""The webhook micro-batch coalescer (include/gkgpu.h coalesce_us):
concurrent single-review Query(violation) calls -- one per admission request in
the reference (pkg/webhook/policy.go:371-387, Client.Review -> Driver.Query,
vendor/.../frameworks/constraint/pkg/client/client.go:763-800) -- are evaluated
together in one launch, and every caller gets exactly its own review's results.

ctypes releases the GIL for the duration of each C call, so these Python
threads really are concurrent callers of gk_query."""
import collections
import json
import threading

import pytest

import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, augmented_review

from parity import engine_rows, oracle_for, oracle_review

VIOLATION = 'hooks["admission.k8s.gatekeeper.sh"].violation'


def _driver(**kw):
    d = gkgpu.Driver(**kw)
    cl = Client(d)
    ts, cs = W.config2()
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    return d, ts, cs


def _race(n, call):
    out, errs = [None] * n, []
    go = threading.Barrier(n)

    def run(i):
        try:
            go.wait()
            out[i] = call(i)
        except Exception as ex:  # noqa: BLE001
            out[i] = ex
    th = [threading.Thread(target=run, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    return out, errs


def test_coalesced_callers_all_get_the_launch_error_without_a_device():
    """Host-only container: the coalesced launch fails (no HIP device); every
    caller of the launch gets the failure with its message, none hangs, and
    the launches served fewer launches than calls."""
    if gkgpu.Driver.device_available():
        pytest.skip("a HIP device is visible: the GPU test covers the coalescer")
    d, _, _ = _driver(coalesce_us=20000, coalesce_max=64)
    pods, ns_of, ns_objs = W.gen_pods(24, seed=3, n_namespaces=4)
    inputs = [json.dumps({"review": augmented_review(p, ns_objs[n])}) for p, n in zip(pods, ns_of)]
    out, _ = _race(len(inputs), lambda i: d.query(VIOLATION, inputs[i]))
    assert all(isinstance(o, RuntimeError) for o in out), out
    assert all("device" in str(o).lower() for o in out), out[0]
    launches, served = d.coalesce_stats()
    assert served == len(inputs)
    assert launches < len(inputs)


@pytest.mark.gpu
def test_one_bad_input_fails_only_its_own_caller():
    """On the device: 32 concurrent coalesced callers, one of them with an
    input that is not JSON.  That caller gets an error; every other caller
    gets exactly the oracle's results for its own review."""
    if not gkgpu.Driver.device_available():
        pytest.fail("no HIP device visible")
    pods, ns_of, ns_objs = W.gen_pods(32, seed=23, n_namespaces=6)
    reviews = [augmented_review(p, ns_objs[n]) for p, n in zip(pods, ns_of)]
    inputs = [json.dumps({"review": rv}) for rv in reviews]
    bad = 9
    inputs[bad] = '{"review": {"object": '
    ts, cs = W.config2()
    od = oracle_for(ts, cs)
    d, _, _ = _driver(coalesce_us=20000, coalesce_max=64)
    out, _ = _race(len(inputs), lambda i: d.query(VIOLATION, inputs[i]))
    assert isinstance(out[bad], RuntimeError), out[bad]
    for i, o in enumerate(out):
        if i == bad:
            continue
        assert not isinstance(o, Exception), (i, o)
        assert not any(o.status), (i, list(o.status))
        assert collections.Counter(engine_rows(o, 1)[0]) == collections.Counter(oracle_review(od, reviews[i])), i
    launches, served = d.coalesce_stats()
    assert served == len(inputs) and launches < served


@pytest.mark.gpu
def test_coalesced_queries_equal_the_oracle():
    """64 concurrent Query(violation) calls with the coalescer on: every result
    set equals the oracle's for that caller's own review, and the calls were
    served by fewer launches than calls.  Also, as references: the same inputs
    as one explicit gk_query_batch, sequential coalesced calls (batches of
    one), and concurrent calls with coalesce_max 1 (concurrent single-review
    launches)."""
    if not gkgpu.Driver.device_available():
        pytest.fail("no HIP device visible")
    pods, ns_of, ns_objs = W.gen_pods(64, seed=17, n_namespaces=8)
    reviews = [augmented_review(p, ns_objs[n]) for p, n in zip(pods, ns_of)]
    inputs = [json.dumps({"review": rv}) for rv in reviews]
    ts, cs = W.config2()
    od = oracle_for(ts, cs)
    want = [collections.Counter(oracle_review(od, rv)) for rv in reviews]

    def check(tag, results):
        bad = []
        for i, res in enumerate(results):
            if isinstance(res, Exception):
                bad.append((i, repr(res)))
                continue
            got = collections.Counter(engine_rows(res, 1)[0]) if all(r.review == 0 for r in res.results) else None
            if any(res.status) or got != want[i]:
                bad.append((i, len(res.results), sum(want[i].values()), list(res.status)))
        return "%s: %d of %d differ %r" % (tag, len(bad), len(results), bad[:4]) if bad else None

    d2, _, _ = _driver()
    batch = engine_rows(d2.query_batch(inputs), len(inputs))
    errs = []
    b = [i for i in range(len(inputs)) if collections.Counter(batch[i]) != want[i]]
    if b:
        errs.append("query_batch: %d differ %r" % (len(b), b[:4]))
    d, _, _ = _driver(coalesce_us=5000, coalesce_max=256)
    errs.append(check("sequential coalesced", [d.query(VIOLATION, x) for x in inputs[:8]]))
    warm = engine_rows(d.query_batch(inputs), len(inputs))  # the same engine, after the calls above
    b = [i for i in range(len(inputs)) if collections.Counter(warm[i]) != want[i]]
    if b:
        errs.append("query_batch on the coalescing engine: %d differ %r" % (len(b), b[:4]))
    d1, _, _ = _driver(coalesce_us=5000, coalesce_max=1)
    out1, _ = _race(len(inputs), lambda i: d1.query(VIOLATION, inputs[i]))
    errs.append(check("concurrent, max 1", out1))
    out, _ = _race(len(inputs), lambda i: d.query(VIOLATION, inputs[i]))
    launches, served = d.coalesce_stats()
    if any(isinstance(o, Exception) or any(o.status) or collections.Counter(engine_rows(o, 1)[0]) != want[i]
           for i, o in enumerate(out)):
        tot_got = sum(len(o.results) for o in out if not isinstance(o, Exception))
        errs.append("coalesced rows %d vs oracle %d; review 0 got %r" % (
            tot_got, sum(sum(w.values()) for w in want), sorted(engine_rows(out[0], 1)[0])[:6]))
    errs.append(check("concurrent coalesced (%d launches for %d calls)" % (launches, served), out))
    errs = [e for e in errs if e]
    assert not errs, errs
    assert served == len(inputs) + 8, (launches, served)
    assert launches < served
