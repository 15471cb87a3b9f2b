"""The boundary's concurrency contract (SURVEY 8(b) "Threading"): the local
driver evaluates under modulesMux.RLock and serializes module changes
(vendor/github.com/open-policy-agent/frameworks/constraint/pkg/client/drivers/
local/local.go:62-68, 117, 303-304).  The engine runs evaluations concurrently,
each on its own evaluation context, and a mutation waits for the evaluations
in flight; every evaluation therefore sees ONE engine state.

ctypes releases the GIL for the duration of every C call, so these Python
threads really do call into the engine at the same time."""
import collections
import json
import random
import threading

import pytest

import gkgpu
from gkgpu import workloads as W
from gkgpu.client import augmented_review, constraint_path

from parity import engine_for, engine_rows, oracle_for, oracle_review


def _limits(cpu, memory):
    return W.constraint("K8sContainerLimits", "container-must-have-limits",
                        match={"kinds": [{"apiGroups": [""], "kinds": ["Pod"]}]},
                        parameters={"cpu": cpu, "memory": memory})


def _inputs(n_batches, per, seed):
    pods, ns_of, ns_objs = W.gen_pods(n_batches * per, seed=seed, n_namespaces=30)
    reviews = [augmented_review(p, ns_objs[n]) for p, n in zip(pods, ns_of)]
    return [reviews[i * per:(i + 1) * per] for i in range(n_batches)]


def _want(templates, constraints, batches):
    od = oracle_for(templates, constraints)
    return [[collections.Counter(oracle_review(od, rv)) for rv in b] for b in batches]


@pytest.mark.gpu
def test_concurrent_queries_see_one_state_while_a_constraint_is_reput():
    """8 threads issue gk_query_batch while a 9th re-puts the container-limits
    constraint with alternating parameters: every batch's results equal the
    oracle's for exactly one of the two constraint sets (no torn evaluation),
    both states are observed, and the generation each result reports names
    the state it saw."""
    if not gkgpu.Driver.device_available():
        pytest.fail("no HIP device visible")
    ts, cs = W.config2()
    state_a = cs
    state_b = [c if c["kind"] != "K8sContainerLimits" else _limits("100m", "512Mi") for c in cs]
    batches = _inputs(8, 48, seed=7)
    want = {"A": _want(ts, state_a, batches), "B": _want(ts, state_b, batches)}
    # the two states must differ on these inputs, or the test proves nothing
    assert want["A"] != want["B"]
    drv = gkgpu.Driver()
    engine_for(drv, ts, state_a)
    inputs = [[json.dumps({"review": rv}) for rv in b] for b in batches]
    drv.query_batch(inputs[0])  # compile the template kernels before the race
    lock = threading.Lock()
    seen = collections.Counter()
    gens = {}
    errors = []
    stop = threading.Event()

    def worker(t):
        rng = random.Random(t)
        try:
            for _ in range(12):
                k = rng.randrange(len(batches))
                res = drv.query_batch(inputs[k])
                got = [collections.Counter(r) for r in engine_rows(res, len(batches[k]))]
                assert not any(res.status), res.status
                which = [s for s in ("A", "B") if got == want[s][k]]
                if not which:
                    bad = [(i, dict(got[i]), dict(want["A"][k][i]), dict(want["B"][k][i]))
                           for i in range(len(got)) if got[i] != want["A"][k][i] and got[i] != want["B"][k][i]]
                    nA = sum(got[i] == want["A"][k][i] for i in range(len(got)))
                    nB = sum(got[i] == want["B"][k][i] for i in range(len(got)))
                    raise AssertionError("batch %d gen %d matches neither constraint set (rows like A %d, like B %d "
                                         "of %d); reviews unlike both: %r" % (k, res.generation, nA, nB, len(got), bad[:2]))
                with lock:
                    seen[which[0]] += 1
                    gens.setdefault(res.generation, set()).add(which[0])
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    def mutator():
        flip = False
        try:
            while not stop.is_set():
                flip = not flip
                c = (state_b if flip else state_a)[2]
                assert c["kind"] == "K8sContainerLimits"
                drv.put_data(constraint_path(c), c)
                stop.wait(0.01)
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    mt = threading.Thread(target=mutator)
    mt.start()
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    stop.set()
    mt.join(timeout=60)
    assert not errors, errors[:3]
    assert sum(seen.values()) == 8 * 12
    assert seen["A"] > 0 and seen["B"] > 0, seen
    # one generation = one state
    assert all(len(v) == 1 for v in gens.values()), gens


def test_concurrent_staging_and_mutation_on_the_host():
    """Host-only engine: threads stage Query inputs (flatten + intern under the
    shared lock) while another thread puts and deletes constraints and synced
    data; nothing deadlocks, every staged batch is complete, and the permanent
    node region stays bounded (replaced documents are compacted)."""
    ts, cs = W.config2()
    drv = gkgpu.Driver(host_only=True)
    engine_for(drv, ts, cs)
    batches = _inputs(4, 32, seed=11)
    inputs = [[json.dumps({"review": rv}) for rv in b] for b in batches]
    errors = []
    stop = threading.Event()

    def stager(t):
        try:
            for i in range(20):
                b = drv.debug_stage_inputs(inputs[(t + i) % len(inputs)])
                assert b.stats()[0] == len(inputs[(t + i) % len(inputs)])
                b.free()
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    def mutator():
        k = 0
        try:
            while not stop.is_set():
                k += 1
                c = _limits("%dm" % (100 + k % 7), "1Gi")
                drv.put_data(constraint_path(c), c)
                drv.put_data("/external/admission.k8s.gatekeeper.sh/namespace/ns%d/v1/Service/s" % (k % 5),
                             {"apiVersion": "v1", "kind": "Service", "metadata": {"name": "s", "namespace": "ns%d" % (k % 5)},
                              "spec": {"selector": {"app": "a%d" % k}}})
                drv.constraints()
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    th = [threading.Thread(target=stager, args=(t,)) for t in range(6)]
    mt = threading.Thread(target=mutator)
    mt.start()
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=240)
    stop.set()
    mt.join(timeout=60)
    assert not errors, errors[:3]
    assert len(drv.constraints()) == len(cs)


def test_inventory_churn_keeps_the_permanent_region_bounded():
    """ADVICE r02 (engine.cc sync_inventory): every inventory rebuild used to
    append a fresh copy of data.inventory to the permanent node region and never
    reclaim the previous one.  Put / delete synced objects repeatedly, with an
    evaluation between (which rebuilds the tree for unique-service-selector's
    join), and check that the region stays within a small multiple of its live
    size."""
    ts, cs = W.config2()
    drv = gkgpu.Driver(host_only=True)
    engine_for(drv, ts, cs)
    batch = [json.dumps({"review": rv}) for rv in _inputs(1, 8, seed=5)[0]]
    svc = lambda i: {"apiVersion": "v1", "kind": "Service",  # noqa: E731
                     "metadata": {"name": "s%d" % i, "namespace": "default"},
                     "spec": {"selector": {"app": "x%d" % i, "tier": "t" * (i % 40)}}}
    path = lambda i: "/external/admission.k8s.gatekeeper.sh/namespace/default/v1/Service/s%d" % i  # noqa: E731
    for i in range(300):
        drv.put_data(path(i), svc(i))
    drv.debug_stage_inputs(batch).free()
    live, _ = drv.debug_store_sizes()
    peak = live
    for r in range(400):
        # a constraint re-put after the tree leaves the old tree behind it
        c = _limits("%dm" % (100 + r % 3), "1Gi")
        drv.put_data(constraint_path(c), c)
        drv.delete_data(path(r % 300))
        drv.put_data(path(r % 300), svc(r % 300 + 1000))
        drv.debug_stage_inputs(batch).free()
        peak = max(peak, drv.debug_store_sizes()[0])
    # garbage is compacted once it outgrows max(2^20 nodes, the live region)
    assert peak <= 2 * live + (1 << 20) + 10000, (live, peak)
    n_end, _ = drv.debug_store_sizes()
    assert n_end < 4 * live + (1 << 20), (live, n_end)
