"""ctypes front of oracle/libgkcpu.so (cpuvm.cc) -- the CPU baseline of the
audit sweep.  TEST / MEASUREMENT INFRASTRUCTURE: only tests/ and bench.py's
cpu_baseline leg use it; it never evaluates anything for the product path.

It runs the engine's compiled template bytecode with the engine's own device
runtime (devrt.h) compiled for the host, on host threads, over a staged batch
whose documents are still in the engine's host arena (gk_debug_host_args).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def lib_path() -> str:
    return os.path.join(_HERE, "libgkcpu.so")


def load():
    global _LIB
    if _LIB is None:
        lib = C.CDLL(lib_path())
        lib.gkcpu_devargs_size.restype = C.c_size_t
        lib.gkcpu_sweep.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_uint64)]
        lib.gkcpu_sweep.restype = C.c_double
        lib.gkcpu_build_joins.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int]
        lib.gkcpu_build_joins.restype = C.c_int
        _LIB = lib
    return _LIB


def _host_args(driver, batch, joins: bool, threads: int, columns: bool = False):
    """the batch's host launch arguments; joins: with the checker's own join
    indexes built from the engine's join plan (cpuvm.cc gkcpu_build_joins),
    else every join site scans; columns: the batch's column form
    (colstore.h), read as the device reads it"""
    lib = load()
    glib = driver._lib
    n = lib.gkcpu_devargs_size()
    buf = (C.c_uint8 * n)()
    fn = glib.gk_debug_host_args_columns if columns else glib.gk_debug_host_args
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]
    driver._check(fn(driver._e, batch._h, buf, n))
    if joins:
        glib.gk_debug_join_plan.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64)]
        sites, ns = C.c_void_p(), C.c_uint64()
        driver._check(glib.gk_debug_join_plan(driver._e, C.byref(sites), C.byref(ns)))
        if ns.value:
            lib.gkcpu_build_joins(buf, sites, ns.value, max(1, threads))
    return buf


def sweep(driver, batch, lo: int = 0, hi=None, threads: int = 1, joins: bool = True):
    """(seconds, evals, violations, message bytes, flagged pairs) of reviews
    [lo, hi) of `batch` x every constraint, on `threads` host threads (the
    join indexes' build not timed)"""
    lib = load()
    buf = _host_args(driver, batch, joins, threads)
    out = (C.c_uint64 * 4)()
    hi = batch.n if hi is None else hi
    s = lib.gkcpu_sweep(buf, lo, hi, threads, out)
    return s, out[0], out[1], out[2], out[3]


def sweep_digest(driver, batch, threads: int = 1, joins: bool = True, columns: bool = False):
    """sweep() over the whole batch plus an order-free digest of every result
    row (oracle/cpuvm.cc gkcpu_sweep_digest): (evals, violations, flagged,
    digest).  row_digest computes the same over rows from elsewhere (the
    oracle), so tests compare rows, not just counts."""
    lib = load()
    lib.gkcpu_sweep_digest.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_uint64)]
    lib.gkcpu_sweep_digest.restype = C.c_double
    buf = _host_args(driver, batch, joins, threads, columns)
    out = (C.c_uint64 * 5)()
    lib.gkcpu_sweep_digest(buf, 0, batch.n, threads, out)
    return out[0], out[1], out[3], out[4]


def device_rows_digest(tuples, raw, threads: int = 8):
    """row_digest of a device evaluation's raw output (DeviceOutput.tuples()
    and .bytes(), host numpy arrays or CPU tensors): (digest, rows hashed),
    computed natively (oracle/cpuvm.cc gkcpu_rows_digest)"""
    import numpy as np
    lib = load()
    lib.gkcpu_rows_digest.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_int,
                                      C.POINTER(C.c_uint64)]
    lib.gkcpu_rows_digest.restype = C.c_uint64
    t = np.ascontiguousarray(np.asarray(tuples, dtype=np.int32))
    b = np.ascontiguousarray(np.asarray(raw, dtype=np.uint8))
    n = C.c_uint64()
    d = lib.gkcpu_rows_digest(t.ctypes.data, t.size // 8, b.ctypes.data, b.size, threads, C.byref(n))
    return int(d), int(n.value)


def row_hash(review: int, constraint: int, msg: bytes, details: bytes) -> int:
    """FNV-1a 64 over (u32 review LE, u32 constraint LE, msg, 0xff, details)"""
    h = 1469598103934665603
    for b in review.to_bytes(4, "little") + constraint.to_bytes(4, "little") + msg + b"\xff" + details:
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def row_digest(rows) -> int:
    """rows: iterable of (review, constraint, msg str, details JSON str)"""
    d = 0
    for rv, c, m, det in rows:
        d = (d + row_hash(rv, c, m.encode("utf-8", "surrogateescape"), det.encode("utf-8", "surrogateescape"))) \
            & 0xFFFFFFFFFFFFFFFF
    return d


def referenced(driver, batch, only: int = -1, lo: int = 0, hi=None, threads: int = 1, pc_hist=None, joins: bool = True):
    """SURVEY 8(d) reference accounting of reviews [lo, hi) x constraint `only`
    (all when < 0): dict(nodes, strings, string_bytes, violations, flagged);
    pc_hist: a ctypes uint64 array of the code size receiving per-instruction
    execution counts (one thread)"""
    lib = load()
    glib = driver._lib
    lib.gkcpu_referenced.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                                     C.POINTER(C.c_uint64), C.c_void_p]
    lib.gkcpu_referenced.restype = C.c_int
    buf = _host_args(driver, batch, joins, threads)
    glib.gk_debug_store_sizes.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    nn, ns = C.c_uint64(), C.c_uint64()
    driver._check(glib.gk_debug_store_sizes(driver._e, C.byref(nn), C.byref(ns)))
    # node ids index the permanent region followed by the batch's documents
    n_nodes = nn.value + batch.stats()[1]
    out = (C.c_uint64 * 5)()
    hi = batch.n if hi is None else hi
    lib.gkcpu_referenced(buf, n_nodes, ns.value, lo, hi, only, threads, out,
                         C.cast(pc_hist, C.c_void_p) if pc_hist is not None else None)
    return {"nodes": out[0], "strings": out[1], "string_bytes": out[2], "violations": out[3], "flagged": out[4]}
