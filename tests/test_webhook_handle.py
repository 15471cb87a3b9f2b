"""Handle's host steps ahead of the engine (gkgpu/webhook.py handle_requests,
pkg/webhook/policy.go:142-223, 363-400), with a stub engine: the
service-account bypass, DELETE reviewing oldObject, the webhook process
excluder, and reviewRequest's Namespace fetch (cached client first, the API
reader only on NotFound, any other error -> 500)."""
import pytest

from gkgpu.driver import Results
from gkgpu.webhook import (ALLOWED, ERROR, NamespaceFetcher, NotFound, gk_service_account, handle_requests,
                           namespace_object)


class StubEngine:
    def __init__(self, excluded=()):
        self.excluded = set(excluded)
        self.inputs = []

    def is_namespace_excluded(self, process, ns):
        return process == "webhook" and ns in self.excluded

    def query_batch(self, inputs):
        self.inputs.extend(inputs)
        return Results([], [0] * len(inputs), [0] * len(inputs), [])


def _req(ns="team-a", kind="Pod", group="", op="CREATE", obj=None, old=None, user="alice"):
    r = {"uid": "u", "kind": {"group": group, "version": "v1", "kind": kind},
         "resource": {"group": group, "version": "v1", "resource": kind.lower() + "s"},
         "operation": op, "userInfo": {"username": user},
         "object": obj if obj is not None else {"kind": kind, "metadata": {"name": "x"}},
         "oldObject": old}
    if ns:
        r["namespace"] = ns
    return r


class Api:
    def __init__(self, cache=(), server=(), cache_error=None):
        self.cache = {n: namespace_object(n) for n in cache}
        self.server = {n: namespace_object(n) for n in server}
        self.cache_error = cache_error
        self.reads = []

    def cache_get(self, name):
        if self.cache_error:
            raise self.cache_error
        if name not in self.cache:
            raise NotFound('namespaces "%s" not found' % name)
        return self.cache[name]

    def reader_get(self, name):
        self.reads.append(name)
        if name not in self.server:
            raise NotFound('namespaces "%s" not found' % name)
        return self.server[name]


def _fetcher(api):
    return NamespaceFetcher(api.cache_get, api.reader_get)


def test_cached_namespace_never_reaches_the_reader():
    api, eng = Api(cache=["team-a"], server=["team-a"]), StubEngine()
    out = handle_requests(eng, [_req("team-a")], _fetcher(api))
    assert out[0].code == ALLOWED and api.reads == []
    import json
    review = json.loads(eng.inputs[0])["review"]
    assert review["_unstable"]["namespace"]["metadata"]["name"] == "team-a"


def test_cache_miss_falls_back_to_the_api_reader():
    api, eng = Api(cache=[], server=["team-b"]), StubEngine()
    out = handle_requests(eng, [_req("team-b")], _fetcher(api))
    assert out[0].code == ALLOWED and api.reads == ["team-b"] and len(eng.inputs) == 1


def test_reader_not_found_and_cache_errors_fail_the_request():
    api, eng = Api(cache=[], server=[]), StubEngine()
    out = handle_requests(eng, [_req("gone")], _fetcher(api))
    assert out[0].code == ERROR and 'namespaces "gone" not found' in out[0].message and eng.inputs == []
    # a cache error other than NotFound does not consult the reader (policy.go:375-377)
    api = Api(cache=[], server=["team-a"], cache_error=RuntimeError("cache unavailable"))
    out = handle_requests(eng, [_req("team-a")], _fetcher(api))
    assert out[0].code == ERROR and out[0].message == "cache unavailable" and api.reads == []


def test_namespace_kind_and_cluster_scoped_requests_fetch_nothing():
    api, eng = Api(), StubEngine()
    out = handle_requests(eng, [_req("team-a", kind="Namespace"), _req(None, kind="ClusterRole", group="rbac")],
                          _fetcher(api))
    assert [o.code for o in out] == [ALLOWED, ALLOWED] and api.reads == []
    import json
    assert [json.loads(x)["review"]["_unstable"] for x in eng.inputs] == [{}, {}]


def test_service_account_delete_and_excluded_namespace():
    api, eng = Api(cache=["team-a", "kube-system"]), StubEngine(excluded=["kube-system"])
    old = {"kind": "Pod", "metadata": {"name": "old"}}
    reqs = [_req(user=gk_service_account()), _req(op="DELETE", old=None), _req(op="DELETE", obj=None, old=old),
            _req("kube-system")]
    out = handle_requests(eng, reqs, _fetcher(api))
    assert out[0].code == ALLOWED and out[0].message == "Gatekeeper does not self-manage"
    assert out[1].code == ERROR and "Kubernetes v1.15.0+" in out[1].message
    assert out[2].code == ALLOWED
    assert out[3].code == ALLOWED and out[3].message == "Namespace is set to be ignored by Gatekeeper config"
    import json
    assert len(eng.inputs) == 1 and json.loads(eng.inputs[0])["review"]["object"] == old


@pytest.mark.parametrize("n", [0, 5])
def test_order_of_responses_follows_requests(n):
    api, eng = Api(cache=["a"], server=["b"]), StubEngine()
    reqs = [_req("a"), _req("missing"), _req("b")] * n
    out = handle_requests(eng, reqs, _fetcher(api))
    assert [o.code for o in out] == [ALLOWED, ERROR, ALLOWED] * n
