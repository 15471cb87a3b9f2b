"""The device-built path layout of a staged batch (csrc/layout.hip,
GKGPU_DEVICE_LAYOUT, default on): the node array and review columns the
kernels read hold the same documents as the host flattener's forms, and the
audit gives the same rows as over the host-built layout (GKGPU_DEVICE_LAYOUT=0)
-- both are checked against the CPU oracle elsewhere (test_gpu_scale.py runs
the bench workloads with the device layout)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _node_form(monkeypatch):
    """these tests are about the node form's layouts (the column form,
    GKGPU_COLUMNS, is checked against it below)"""
    monkeypatch.setenv("GKGPU_COLUMNS", "0")


def _driver(cfg):
    import gkgpu
    from gkgpu import workloads as W
    from gkgpu.client import Client
    if not gkgpu.Driver.device_available():
        pytest.fail("no HIP device visible")
    d = gkgpu.Driver()
    cl = Client(d)
    ts, cs = getattr(W, "config%d" % cfg)()
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    return d


def _rows(res):
    return sorted((r.review, r.constraint, r.msg, r.details_json, r.enforcement_action) for r in res.results)


@pytest.mark.parametrize("cfg,n", [(2, 30000), (4, 20000), (3, 20000)])
def test_device_layout_holds_the_host_documents(cfg, n, monkeypatch):
    from gkgpu import workloads as W
    from gkgpu.page import Page
    d = _driver(cfg)
    d.excluder_add(["audit"], ["ns-0003", "c4-ns-0002"])
    objs, nss = getattr(W, "gen_pods_json" if cfg == 2 else "gen_config%d_json" % cfg)(n)
    pg = Page.from_lists(objs, nss)
    host = d.debug_flatten(pg, 4)[0]
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("GKGPU_DEVICE_LAYOUT", mode)
        b = d.stage_page(pg)
        assert d.debug_batch_hash(b) == host, mode
        res = b.eval(decode=True, with_status=True)
        out[mode] = (_rows(res), list(res.status), list(res.totals))
        b.free()
    assert out["1"] == out["0"]
    assert len(out["1"][0]) > 0
    # the column form of the same page (colstore.h): the same rows
    monkeypatch.setenv("GKGPU_COLUMNS", "1")
    b = d.stage_page(pg)
    assert b.columnar(), b.columns_why()
    res = b.eval(decode=True, with_status=True)
    assert (_rows(res), list(res.status), list(res.totals)) == out["1"]
    b.free()
