"""The benchmark's native admission load generator (libgkload.so,
gatekeeper-1_amd/csrc/loadgen.cc): open-loop single-review gk_query calls
from C++ threads through the C ABI.  CPU: the library loads, every scheduled
request gets a latency, and a failing engine call surfaces as the status.
GPU: the coalesced calls all succeed and the coalescer served them."""
import ctypes as C
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd")]
VIOL = b'hooks["admission.k8s.gatekeeper.sh"].violation'


def _lib():
    lib = C.CDLL(os.path.join(ROOT, "gatekeeper-1_amd", "gkgpu", "libgkload.so"))
    lib.gkload_open_loop.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t,
                                     C.c_size_t, C.c_int, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
    return lib


def _run(drv, inputs, n, clients, rate):
    blobs = [(x if isinstance(x, str) else json.dumps(x)).encode() for x in inputs]
    arr = (C.c_char_p * len(blobs))(*blobs)
    lens = (C.c_size_t * len(blobs))(*[len(b) for b in blobs])
    lat = (C.c_double * n)(*([-1.0] * n))
    el = C.c_double()
    rc = _lib().gkload_open_loop(drv._e, VIOL, arr, lens, len(blobs), n, clients, rate, lat, C.byref(el))
    return rc, list(lat), el.value


def _driver(**kw):
    import gkgpu
    from gkgpu import workloads as W
    from gkgpu.client import Client
    ts, cs = W.config5(5)
    d = gkgpu.Driver(**kw)
    cl = Client(d)
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    return d, W.gen_admission_inputs(32, seed=99)


def test_loadgen_schedules_every_request_and_reports_failures():
    d, ins = _driver(host_only=True)
    rc, lat, el = _run(d, ins, 12, 3, 2000.0)
    assert rc != 0  # no device: every gk_query fails, the status comes back
    assert all(x >= 0 for x in lat) and el > 0
    assert _lib().gkload_open_loop(None, VIOL, None, None, 0, 0, 1, 1.0, None, None) != 0
    d.close()


@pytest.mark.gpu
def test_loadgen_coalesced_calls_succeed():
    d, ins = _driver(coalesce_us=300, coalesce_max=256)
    b0, r0 = d.coalesce_stats()
    rc, lat, el = _run(d, ins, 256, 16, 5000.0)
    b1, r1 = d.coalesce_stats()
    assert rc == 0
    assert all(x >= 0 for x in lat) and el > 0
    assert r1 - r0 == 256 and b1 - b0 < 256
    d.close()


def _batch_loop(drv, inputs, batch, steps):
    lib = _lib()
    lib.gkload_batch_loop.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t,
                                      C.c_size_t, C.c_size_t, C.POINTER(C.c_double), C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    blobs = [(x if isinstance(x, str) else json.dumps(x)).encode() for x in inputs]
    arr = (C.c_char_p * len(blobs))(*blobs)
    lens = (C.c_size_t * len(blobs))(*[len(b) for b in blobs])
    lat = (C.c_double * steps)()
    rows, nb, fl = C.c_uint64(), C.c_uint64(), C.c_uint64()
    rc = lib.gkload_batch_loop(drv._e, arr, lens, len(blobs) // batch, batch, steps, lat, C.byref(rows), C.byref(nb),
                               C.byref(fl))
    return rc, list(lat), rows.value, nb.value, fl.value


def test_batch_loop_reports_failures():
    d, ins = _driver(host_only=True)
    rc, _lat, _r, _b, _f = _batch_loop(d, ins, 16, 2)
    assert rc != 0
    d.close()


@pytest.mark.gpu
def test_batch_loop_rows_equal_query_batch():
    d, ins = _driver()
    rc, lat, rows, nbytes, fl = _batch_loop(d, ins, 16, 4)
    assert rc == 0 and all(x > 0 for x in lat) and fl == 0
    want = len(d.query_batch(ins[:16]).results) + len(d.query_batch(ins[16:32]).results)
    assert rows == 2 * want and nbytes > 0
    d.close()
