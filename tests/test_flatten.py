"""Host flattener (csrc/flatten.cc) and process excluder, on the CPU: the
parallel flattening is content-identical at every thread count, the bulk page
and char** forms agree, and the excluder mirrors excluder.go."""
import json

import pytest

import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client
from gkgpu.page import NO_NS, Page


@pytest.fixture(scope="module")
def drv():
    d = gkgpu.Driver(jit=False)
    cl = Client(d)
    ts, cs = W.config2()
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    return d


def test_flatten_same_content_at_every_thread_count(drv):
    objs, nss = W.gen_pods_json(9000, seed=42, n_namespaces=50)
    pg = Page.from_lists(objs, nss)
    hashes = {drv.debug_flatten(pg, t)[0] for t in (1, 2, 3, 8)}
    assert len(hashes) == 1


def test_path_layout_keeps_every_document(drv):
    """The staged-batch form (flatten.h path-grouped layout: review roots, the
    Namespace documents, then one region of member runs per document path, in
    evaluation order) holds the same documents, columns and node count as the
    per-document layout, at every thread count."""
    objs, nss = W.gen_pods_json(9000, seed=42, n_namespaces=50)
    pg = Page.from_lists(objs, nss)
    # (every part parses its own copy of a Namespace document: node counts
    # depend on the thread count, the same in both layouts)
    for t in (1, 3, 8):
        assert drv.debug_flatten(pg, t)[:2] == drv.debug_flatten(pg, -t)[:2]
    assert len({drv.debug_flatten(pg, -t)[0] for t in (1, 2, 8)}) == 1
    objs, nss = W.gen_config4_json(6000, seed=99)
    pg = Page.from_lists(objs, nss)
    assert drv.debug_flatten(pg, 2)[:2] == drv.debug_flatten(pg, -2)[:2]


def test_path_layout_evaluates_like_the_document_layout(monkeypatch):
    """The engine's programs on the host runtime (oracle/cpuvm.cc) give the same
    violations and message bytes over a batch staged in the path-grouped layout
    as over the same batch staged per document (GKGPU_PATH_LAYOUT=0)."""
    from oracle import cpu_baseline
    d = gkgpu.Driver(host_only=True)
    cl = Client(d)
    ts, cs = W.config2()
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    objs, nss = W.gen_pods_json(12000, seed=5, n_namespaces=40)
    pg = Page.from_lists(objs, nss)
    out = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("GKGPU_PATH_LAYOUT", mode)
        b = d.stage_page(pg)
        out[mode] = cpu_baseline.sweep(d, b, threads=4)[1:]
        b.free()
    assert out["0"] == out["1"]
    assert out["1"][1] > 10000 and out["1"][3] == 0


def test_flatten_mixed_kinds_cluster_scoped_and_escapes(drv):
    objs, nss = W.gen_config4_json(6000, seed=1234)
    objs.append('{"apiVersion":"v1","kind":"ConfigMap","metadata":{"name":"esc\\u00e9\\n\\"q\\"","namespace":"c4-ns-0001"},'
                '"data":{"k":"v","k":"dup-last-wins"}}')
    nss.append(nss[0])
    pg = Page.from_lists(objs, nss)
    h1, n1, _, _ = drv.debug_flatten(pg, 1)
    h8, n8, _, _ = drv.debug_flatten(pg, 8)
    assert h1 == h8 and n1 > 0


def test_flatten_rejects_bad_json(drv):
    pg = Page.from_lists(['{"a": 1}', '{"a": }'], [None, None])
    with pytest.raises(RuntimeError, match="invalid object JSON at 1"):
        drv.debug_flatten(pg, 2)


def test_page_from_lists_shares_namespaces():
    ns = W.namespace_obj("a")
    pg = Page.from_lists([{"k": 1}, {"k": 2}, {"k": 3}], [ns, None, ns])
    assert pg.n == 3 and pg.n_ns == 1
    assert list(pg.obj_ns) == [0, NO_NS, 0]
    assert json.loads(pg.nss) == ns
    assert pg.objs[int(pg.obj_offs[1]):int(pg.obj_offs[2])] == b'{"k":2}'


def test_excluder_mirrors_excluder_go():
    d = gkgpu.Driver(jit=False)
    d.excluder_add(["audit"], ["kube-system"])
    d.excluder_add(["*"], ["gatekeeper-system"])
    assert d.is_namespace_excluded("audit", "kube-system")
    assert not d.is_namespace_excluded("webhook", "kube-system")
    for p in ("audit", "webhook", "sync"):
        assert d.is_namespace_excluded(p, "gatekeeper-system")
    assert not d.is_namespace_excluded("*", "gatekeeper-system")
    d.excluder_clear()
    assert not d.is_namespace_excluded("audit", "kube-system")


def test_excluded_objects_carry_no_document(drv):
    objs, nss = W.gen_pods_json(3000, seed=1, n_namespaces=20)
    pg = Page.from_lists(objs, nss)
    _, n_all, _, _ = drv.debug_flatten(pg, 4)
    drv.excluder_add(["audit"], ["production"])
    try:
        _, n_ex, _, _ = drv.debug_flatten(pg, 4)
    finally:
        drv.excluder_clear()
    assert n_ex < n_all


def test_unparsable_api_version_gives_an_empty_gvk():
    """schema.ParseGroupVersion fails on more than one '/', and
    unstructured.GroupVersionKind() then returns an EMPTY GVK
    (k8s.io/apimachinery unstructured.go:425-432): review.kind is all "" --
    kind included -- in the native flattener, in the Python envelope the
    oracle is fed, and in HandleViolation's resource identity."""
    from gkgpu.client import augmented_review
    obj = {"apiVersion": "a/b/c", "kind": "Pod", "metadata": {"name": "p", "namespace": "n"}}
    assert augmented_review(obj, None)["kind"] == {"group": "", "version": "", "kind": ""}
    ok = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": "d", "namespace": "n"}}
    assert augmented_review(ok, None)["kind"] == {"group": "apps", "version": "v1", "kind": "Deployment"}
    d = gkgpu.Driver(host_only=True)
    b = d.stage_objects([obj, ok], [None, None])
    assert b.resource(0) == ("", "", "p", "n")
    assert b.resource(1) == ("apps/v1", "Deployment", "d", "n")


def test_device_layout_input_holds_the_same_documents(drv, monkeypatch):
    """The per-document arena the device layout pass (layout.hip) permutes --
    containers carrying their document path, shared Namespace runs flagged --
    holds the same documents and columns as both host layouts."""
    for gen, n in ((lambda: W.gen_pods_json(9000, seed=42, n_namespaces=50), 9000),
                   (lambda: W.gen_config4_json(6000, seed=99), 6000)):
        objs, nss = gen()
        pg = Page.from_lists(objs, nss)
        for t in (1, 3):
            monkeypatch.delenv("GKGPU_DEBUG_DEVICE_FORM", raising=False)
            host = drv.debug_flatten(pg, -t)[0]
            monkeypatch.setenv("GKGPU_DEBUG_DEVICE_FORM", "1")
            assert drv.debug_flatten(pg, -t)[0] == host == drv.debug_flatten(pg, t)[0]
