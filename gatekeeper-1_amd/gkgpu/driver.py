"""ctypes binding of the gkgpu C ABI (include/gkgpu.h).

Each method cites the drivers.Driver method it implements
(vendor/github.com/open-policy-agent/frameworks/constraint/pkg/client/drivers/interface.go).
"""
from __future__ import annotations

import ctypes as C
import json
import os
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

GK_REVIEW_ERROR = 1
GK_REVIEW_FALLBACK = 2

TARGET = "admission.k8s.gatekeeper.sh"

EXPORTS = [
    "gk_engine_create", "gk_engine_destroy", "gk_last_error", "gk_device_available", "gk_init", "gk_put_module",
    "gk_put_modules", "gk_delete_module", "gk_delete_modules", "gk_put_data", "gk_delete_data", "gk_query", "gk_dump",
    "gk_free_string", "gk_query_batch", "gk_review_objects", "gk_batch_stage_objects", "gk_batch_eval",
    "gk_batch_free", "gk_batch_device_bytes", "gk_results_count", "gk_results_get", "gk_results_reviews",
    "gk_results_review_status", "gk_results_review_reason", "gk_results_constraints", "gk_results_constraint_total",
    "gk_results_timing", "gk_results_free", "gk_template_status", "gk_constraint_count", "gk_constraint_info",
    "gk_batch_stats", "gk_results_device_counts", "gk_results_copy_status", "gk_results_flag_counts",
    "gk_results_launches", "gk_results_launch", "gk_template_backend", "gk_results_copy_device_output",
    "gk_review_page", "gk_batch_stage_page", "gk_batch_timing", "gk_batch_excluded", "gk_batch_resource",
    "gk_excluder_add", "gk_excluder_clear", "gk_excluder_is_excluded", "gk_results_excluded",
    "gk_batch_eval_audit", "gk_results_sample_count", "gk_results_sample_get", "gk_results_constraint_action",
    "gk_results_export", "gk_results_samples_export", "gk_results_generation", "gk_coalesce_stats",
    "gk_template_joins", "gk_join_stats", "gk_engine_prepare", "gk_audit_cache_sample",
]


class _SampleView(C.Structure):
    _fields_ = [("review", C.c_uint32), ("constraint", C.c_uint32), ("seq", C.c_uint16), ("rule", C.c_uint16),
                ("msg_len", C.c_uint32), ("msg", C.c_void_p), ("msg_stored", C.c_size_t),
                ("enforcement_action", C.c_char_p)]

GK_REVIEW_EXCLUDED = 4
RESOURCE_FIELD = 512


class _Resource(C.Structure):
    _fields_ = [("api_version", C.c_char * RESOURCE_FIELD), ("kind", C.c_char * RESOURCE_FIELD),
                ("name", C.c_char * RESOURCE_FIELD), ("namespace", C.c_char * RESOURCE_FIELD)]


class EngineUnavailable(RuntimeError):
    pass


class QueryError(RuntimeError):
    pass


class _View(C.Structure):
    _fields_ = [
        ("review", C.c_uint32), ("constraint", C.c_uint32), ("constraint_kind", C.c_char_p),
        ("constraint_name", C.c_char_p), ("msg", C.c_void_p), ("msg_len", C.c_size_t),
        ("details_json", C.c_void_p), ("details_len", C.c_size_t), ("enforcement_action", C.c_char_p),
    ]


def lib_path() -> str:
    return os.environ.get("GKGPU_LIB", os.path.join(_HERE, "libgkgpu.so"))


def _one_hip_runtime():
    """PyTorch-ROCm bundles its own HIP runtime, loaded under the file name
    libamdhip64.so; the engine links libamdhip64.so.7 from /opt/rocm.  Loaded
    engine-first, a process later importing torch gets a second HIP/HSA
    runtime, and torch then sees no GPU ("No HIP GPUs are available").  Loaded
    torch-first, the engine's NEEDED libamdhip64.so.7 matches the SONAME torch
    already loaded and there is one runtime.  The engine hands device buffers to
    torch tensors (DeviceOutput, the RCCL exchange), so torch goes first when it
    is installed (GKGPU_NO_TORCH=1 skips it)."""
    if os.environ.get("GKGPU_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load_library():
    global _LIB
    if _LIB is not None:
        return _LIB
    p = lib_path()
    if not os.path.exists(p):
        raise EngineUnavailable("libgkgpu.so not built (%s); run __graft_entry__.build()" % p)
    _one_hip_runtime()
    # template-kernel code objects (jit.cc): the in-tree cache travels with the
    # tree to the GPU box, so a fresh process there loads them instead of
    # compiling every template with hipRTC again
    tree_cache = os.path.join(os.path.dirname(os.path.dirname(_HERE)), ".jitcache")
    if "GKGPU_JIT_CACHE" not in os.environ and os.path.isdir(tree_cache) and os.access(tree_cache, os.W_OK):
        os.environ["GKGPU_JIT_CACHE"] = tree_cache
    lib = C.CDLL(p)
    vp = C.c_void_p
    sz = C.c_size_t
    cp = C.c_char_p
    ppc = C.POINTER(C.c_char_p)
    psz = C.POINTER(C.c_size_t)
    lib.gk_engine_create.argtypes = [cp, C.POINTER(vp)]
    lib.gk_engine_destroy.argtypes = [vp]
    lib.gk_last_error.argtypes = [vp]
    lib.gk_last_error.restype = cp
    lib.gk_device_available.restype = C.c_int
    lib.gk_init.argtypes = [vp]
    lib.gk_put_module.argtypes = [vp, cp, cp, sz]
    lib.gk_put_modules.argtypes = [vp, cp, ppc, psz, sz]
    lib.gk_delete_module.argtypes = [vp, cp, C.POINTER(C.c_int)]
    lib.gk_delete_modules.argtypes = [vp, cp, C.POINTER(C.c_int)]
    lib.gk_put_data.argtypes = [vp, cp, cp, sz]
    lib.gk_delete_data.argtypes = [vp, cp, C.POINTER(C.c_int)]
    lib.gk_query.argtypes = [vp, cp, cp, sz, C.POINTER(vp)]
    lib.gk_dump.argtypes = [vp, C.POINTER(vp)]
    lib.gk_free_string.argtypes = [vp]
    lib.gk_query_batch.argtypes = [vp, ppc, psz, sz, C.POINTER(vp)]
    lib.gk_coalesce_stats.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    lib.gk_review_objects.argtypes = [vp, ppc, psz, ppc, psz, sz, C.POINTER(vp)]
    lib.gk_batch_stage_objects.argtypes = [vp, ppc, psz, ppc, psz, sz, C.POINTER(vp)]
    lib.gk_batch_eval.argtypes = [vp, vp, C.c_int, C.POINTER(vp)]
    lib.gk_batch_free.argtypes = [vp]
    lib.gk_batch_device_bytes.argtypes = [vp]
    lib.gk_batch_device_bytes.restype = C.c_uint64
    lib.gk_results_count.argtypes = [vp]
    lib.gk_results_count.restype = sz
    lib.gk_results_get.argtypes = [vp, sz, C.POINTER(_View)]
    lib.gk_results_export.argtypes = [vp, vp, sz, C.POINTER(sz)]
    lib.gk_results_samples_export.argtypes = [vp, vp, sz, C.POINTER(sz)]
    lib.gk_results_reviews.argtypes = [vp]
    lib.gk_results_reviews.restype = sz
    lib.gk_results_review_status.argtypes = [vp, sz]
    lib.gk_results_review_status.restype = C.c_uint32
    lib.gk_results_review_reason.argtypes = [vp, sz]
    lib.gk_results_review_reason.restype = C.c_uint32
    lib.gk_results_constraints.argtypes = [vp]
    lib.gk_results_constraints.restype = sz
    lib.gk_results_constraint_total.argtypes = [vp, sz]
    lib.gk_results_constraint_total.restype = C.c_uint64
    lib.gk_results_timing.argtypes = [vp, C.POINTER(C.c_double)]
    lib.gk_results_generation.argtypes = [vp]
    lib.gk_results_generation.restype = C.c_uint64
    lib.gk_results_free.argtypes = [vp]
    pu64 = C.POINTER(C.c_uint64)
    lib.gk_batch_stats.argtypes = [vp, pu64, pu64, pu64, pu64]
    lib.gk_results_device_counts.argtypes = [vp, pu64, pu64]
    lib.gk_results_copy_status.argtypes = [vp, C.c_void_p, C.c_void_p]
    lib.gk_results_flag_counts.argtypes = [vp, pu64, pu64]
    lib.gk_results_launches.argtypes = [vp]
    lib.gk_results_launches.restype = sz
    lib.gk_results_launch.argtypes = [vp, sz, C.POINTER(cp), C.POINTER(C.c_double), C.POINTER(C.c_uint32), pu64, pu64]
    lib.gk_template_backend.argtypes = [vp, cp, C.POINTER(C.c_int), C.POINTER(cp)]
    lib.gk_template_joins.argtypes = [vp, cp, C.POINTER(cp)]
    lib.gk_template_joins.restype = C.c_int
    u64p = C.POINTER(C.c_uint64)
    lib.gk_join_stats.argtypes = [vp, u64p, u64p, u64p, u64p, C.POINTER(C.c_double)]
    lib.gk_results_copy_device_output.argtypes = [vp, vp, vp, vp, C.POINTER(C.c_uint64)]
    lib.gk_results_vm_profile.argtypes = [vp, C.c_void_p, sz]
    lib.gk_results_vm_profile.restype = sz
    lib.gk_template_status.argtypes = [vp, cp, C.POINTER(cp)]
    lib.gk_template_status.restype = C.c_int
    lib.gk_constraint_count.argtypes = [vp]
    lib.gk_constraint_count.restype = sz
    lib.gk_constraint_info.argtypes = [vp, sz, C.POINTER(cp), C.POINTER(cp)]
    page_args = [vp, C.c_char_p, vp, sz, C.c_char_p, vp, sz, vp]
    lib.gk_review_page.argtypes = page_args + [C.POINTER(vp)]
    lib.gk_batch_stage_page.argtypes = page_args + [C.POINTER(vp)]
    lib.gk_debug_flatten_page.argtypes = page_args + [C.c_int, pu64, pu64, C.POINTER(C.c_double)]
    lib.gk_batch_timing.argtypes = [vp, C.POINTER(C.c_double)]
    lib.gk_batch_excluded.argtypes = [vp]
    lib.gk_batch_excluded.restype = C.c_uint64
    lib.gk_batch_resource.argtypes = [vp, vp, sz, C.POINTER(_Resource)]
    lib.gk_excluder_add.argtypes = [vp, ppc, sz, ppc, sz]
    lib.gk_excluder_clear.argtypes = [vp]
    lib.gk_excluder_is_excluded.argtypes = [vp, cp, cp]
    lib.gk_results_excluded.argtypes = [vp]
    lib.gk_results_excluded.restype = C.c_uint64
    lib.gk_batch_eval_audit.argtypes = [vp, vp, C.c_uint32, C.POINTER(vp)]
    lib.gk_results_sample_count.argtypes = [vp]
    lib.gk_results_sample_count.restype = sz
    lib.gk_results_sample_get.argtypes = [vp, sz, C.POINTER(_SampleView)]
    lib.gk_results_constraint_action.argtypes = [vp, sz]
    lib.gk_results_constraint_action.restype = cp
    _LIB = lib
    return lib


def _b(s) -> bytes:
    return s.encode("utf-8", "surrogateescape") if isinstance(s, str) else s


@dataclass
class Result:
    """One types.Result (vendor/.../frameworks/constraint/pkg/types/validation.go:11-29)."""
    review: int
    constraint: int
    constraint_kind: str
    constraint_name: str
    msg: str
    details_json: str
    enforcement_action: str
    resource: Optional[dict] = None  # HandleViolation's Result.Resource (Client.review sets it)


@dataclass
class Launch:
    kernel: str        # "audit_kernel" (bytecode VM) or "gk_t_<hash>" (template kernel)
    ms: float          # HIP-event duration
    constraints: int   # constraints the launch evaluated
    tuples: int        # violation tuples it wrote
    bytes: int         # message/details bytes it wrote

    def __iter__(self):  # (kernel, ms, constraints) unpacking
        return iter((self.kernel, self.ms, self.constraints))


@dataclass
class Results:
    results: List[Result]
    status: List[int]          # per review: GK_REVIEW_ERROR / GK_REVIEW_FALLBACK bits
    reason: List[int]
    totals: List[int]          # per constraint (device counters)
    timing_ms: List[float] = field(default_factory=list)  # flatten, upload, kernel, download, decode
    device_tuples: int = 0      # violation tuples the kernel wrote (32 B each)
    device_bytes: int = 0       # message/details bytes the kernel wrote
    n_errors: int = 0
    n_fallbacks: int = 0
    vm_profile: List[int] = field(default_factory=list)  # GKGPU_PROFILE=1 diagnostics
    launches: List["Launch"] = field(default_factory=list)  # per kernel launch, in order
    generation: int = 0        # engine state evaluated (gk_results_generation)

    def vm_stats(self):
        """per constraint: (sum VM steps, max lane steps, lanes run, sum of per-wave max steps)"""
        p = self.vm_profile
        return [tuple(p[i:i + 4]) for i in range(0, len(p), 4)]

    def for_review(self, i):
        return [r for r in self.results if r.review == i]


def _vm_profile(lib, h):
    n = lib.gk_results_vm_profile(h, None, 0)
    if not n:
        return []
    buf = (C.c_uint64 * n)()
    lib.gk_results_vm_profile(h, buf, n)
    return list(buf)


def _launches(lib, h):
    out = []
    for i in range(lib.gk_results_launches(h)):
        k, ms, n, t, b = C.c_char_p(), C.c_double(), C.c_uint32(), C.c_uint64(), C.c_uint64()
        lib.gk_results_launch(h, i, C.byref(k), C.byref(ms), C.byref(n), C.byref(t), C.byref(b))
        out.append(Launch(k.value.decode(), ms.value, n.value, t.value, b.value))
    return out


@dataclass
class Sample:
    """one of the first `limit` results of a constraint (gk_sample_view)"""
    review: int
    constraint: int
    seq: int
    rule: int               # 0xffff = autoreject
    msg_len: int            # full message length in bytes
    msg: bytes              # its first min(msg_len, 256) bytes
    enforcement_action: str


@dataclass
class AuditSweep:
    """gk_batch_eval_audit: what one audit sweep hands the status writer"""
    totals: List[int]       # per constraint, over the reviews the engine answered
    samples: List[Sample]   # first `limit` per constraint, evaluation order
    actions: List[str]      # per constraint enforcementAction
    n_errors: int
    n_fallbacks: int
    excluded: int
    timing_ms: List[float]
    device_tuples: int
    device_bytes: int
    launches: List["Launch"]
    # batch indices of the reviews flagged GK_REVIEW_ERROR / GK_REVIEW_FALLBACK:
    # left out of totals and samples (the reference answers them on CPU OPA);
    # AuditWriter.from_sweep / parallel.exchange_audit merge their results in
    flagged: List[int] = field(default_factory=list)


def _collect_audit(lib, h) -> AuditSweep:
    try:
        nc = lib.gk_results_constraints(h)
        totals = [lib.gk_results_constraint_total(h, i) for i in range(nc)]
        actions = [(lib.gk_results_constraint_action(h, i) or b"").decode("utf-8", "surrogateescape") for i in range(nc)]
        # one bulk copy of the samples (gk_results_samples_export) instead of
        # a ctypes call per sample
        import struct
        samples = []
        need = C.c_size_t()
        lib.gk_results_samples_export(h, None, 0, C.byref(need))
        if need.value:
            buf = C.create_string_buffer(need.value)
            lib.gk_results_samples_export(h, buf, need.value, C.byref(need))
            raw = buf.raw
            i = 0
            while i < need.value:
                rv, c, seq, rule, ml, st = struct.unpack_from("<IIHHII", raw, i)
                i += 20
                samples.append(Sample(rv, c, seq, rule, ml, raw[i:i + st], actions[c] if c < nc else ""))
                i += st
        t = (C.c_double * 5)()
        lib.gk_results_timing(h, t)
        dt, db = C.c_uint64(), C.c_uint64()
        lib.gk_results_device_counts(h, C.byref(dt), C.byref(db))
        ne, nf = C.c_uint64(), C.c_uint64()
        lib.gk_results_flag_counts(h, C.byref(ne), C.byref(nf))
        flagged = []
        if ne.value or nf.value:
            import numpy as np
            nr = lib.gk_results_reviews(h)
            st = np.zeros(max(nr, 1), dtype=np.uint32)
            lib.gk_results_copy_status(h, st.ctypes.data, None)
            flagged = np.nonzero(st[:nr] & (GK_REVIEW_ERROR | GK_REVIEW_FALLBACK))[0].tolist()
        return AuditSweep(totals, samples, actions, ne.value, nf.value, lib.gk_results_excluded(h), list(t), dt.value,
                          db.value, _launches(lib, h), flagged)
    finally:
        lib.gk_results_free(h)


def _collect_light(lib, h, with_status: bool = False) -> Results:
    """totals, counters and flag counts only (no result rows; the per-review
    status words as a numpy uint32 array when with_status)."""
    try:
        status = []
        if with_status:
            import numpy as np
            nr = lib.gk_results_reviews(h)
            status = np.zeros(max(nr, 1), dtype=np.uint32)[:nr]
            if nr:
                lib.gk_results_copy_status(h, status.ctypes.data, None)
        nc = lib.gk_results_constraints(h)
        totals = [lib.gk_results_constraint_total(h, i) for i in range(nc)]
        t = (C.c_double * 5)()
        lib.gk_results_timing(h, t)
        dt, db = C.c_uint64(), C.c_uint64()
        lib.gk_results_device_counts(h, C.byref(dt), C.byref(db))
        ne, nf = C.c_uint64(), C.c_uint64()
        lib.gk_results_flag_counts(h, C.byref(ne), C.byref(nf))
        return Results([], status, [], totals, list(t), dt.value, db.value, ne.value, nf.value, _vm_profile(lib, h),
                       _launches(lib, h), lib.gk_results_generation(h))
    finally:
        lib.gk_results_free(h)


def _collect(lib, h, decode=True) -> Results:
    try:
        n = lib.gk_results_count(h)
        out = []
        v = _View()
        for i in range(n):
            lib.gk_results_get(h, i, C.byref(v))
            msg = C.string_at(v.msg, v.msg_len).decode("utf-8", "surrogateescape") if v.msg_len else ""
            det = C.string_at(v.details_json, v.details_len).decode("utf-8", "surrogateescape") if v.details_len else ""
            out.append(Result(v.review, v.constraint, v.constraint_kind.decode(), v.constraint_name.decode(), msg, det,
                              v.enforcement_action.decode()))
        nr = lib.gk_results_reviews(h)
        st = (C.c_uint32 * nr)()
        rs = (C.c_uint32 * nr)()
        lib.gk_results_copy_status(h, st, rs)
        status = list(st)
        reason = list(rs)
        nc = lib.gk_results_constraints(h)
        totals = [lib.gk_results_constraint_total(h, i) for i in range(nc)]
        t = (C.c_double * 5)()
        lib.gk_results_timing(h, t)
        dt, db = C.c_uint64(), C.c_uint64()
        lib.gk_results_device_counts(h, C.byref(dt), C.byref(db))
        return Results(out, status, reason, totals, list(t), dt.value, db.value,
                       sum(1 for x in status if x & 1), sum(1 for x in status if x & 2), _vm_profile(lib, h),
                       _launches(lib, h), lib.gk_results_generation(h))
    finally:
        lib.gk_results_free(h)


def _arr(strings: Sequence):
    bs = [_b(s) if s is not None else None for s in strings]
    arr = (C.c_char_p * len(bs))(*bs)
    lens = (C.c_size_t * len(bs))(*[len(x) if x is not None else 0 for x in bs])
    return arr, lens, bs


class Batch:
    """A device-resident set of reviews (gk_batch_*)."""

    def __init__(self, drv, handle, n):
        self._drv = drv
        self._h = handle
        self.n = n

    def eval(self, decode=True, light=False, device_out=None, with_status=False) -> Results:
        """device_out(n_tuples, n_bytes) -> (tuples_ptr, bytes_ptr): device
        buffers (e.g. torch tensors' data_ptr()) that receive the call's raw
        output (gk_viol records of the reviews the engine answered + message
        bytes) before the handle is freed; device_out.copied(n) is then told
        how many records were written, if it has that method."""
        lib = self._drv._lib
        out = C.c_void_p()
        rc = lib.gk_batch_eval(self._drv._e, self._h, 1 if decode else 0, C.byref(out))
        self._drv._check(rc)
        if device_out is not None:
            dt, db = C.c_uint64(), C.c_uint64()
            lib.gk_results_device_counts(out, C.byref(dt), C.byref(db))
            tp, bp = device_out(dt.value, db.value)
            kept = C.c_uint64()
            rc = lib.gk_results_copy_device_output(self._drv._e, out, tp, bp, C.byref(kept))
            if rc != 0:
                lib.gk_results_free(out)
                self._drv._check(rc)
            if hasattr(device_out, "copied"):
                device_out.copied(kept.value)
        return _collect_light(lib, out, with_status) if light else _collect(lib, out)

    def eval_audit(self, limit: int = 20) -> AuditSweep:
        """one audit sweep: exact totals + first `limit` results per constraint
        (gk_batch_eval_audit; pkg/audit/manager.go:462-508)"""
        lib = self._drv._lib
        out = C.c_void_p()
        self._drv._check(lib.gk_batch_eval_audit(self._drv._e, self._h, limit, C.byref(out)))
        return _collect_audit(lib, out)

    def device_bytes(self) -> int:
        return self._drv._lib.gk_batch_device_bytes(self._h)

    def _columns(self):
        lib = self._drv._lib
        lib.gk_batch_columns.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                         C.POINTER(C.c_uint64)]
        sch, why, nb = C.c_char_p(), C.c_char_p(), C.c_uint64()
        form = lib.gk_batch_columns(self._h, C.byref(sch), C.byref(why), C.byref(nb))
        dec = lambda b: (b or b"").decode("utf-8", "replace")  # noqa: E731
        return form == 1, dec(sch.value), dec(why.value), nb.value

    def columnar(self) -> bool:
        """staged in column form (csrc/colstore.h), not as document nodes"""
        return self._columns()[0]

    def columns_why(self) -> str:
        """why the node form was kept (empty in column form)"""
        return self._columns()[2]

    def columns_schema(self) -> str:
        """the column form's path schema (diagnostics)"""
        return self._columns()[1]

    def timing_ms(self):
        """host staging milliseconds: (parse + build documents, flatten total, upload)"""
        t = (C.c_double * 3)()
        self._drv._lib.gk_batch_timing(self._h, t)
        return tuple(t)

    def excluded(self) -> int:
        return self._drv._lib.gk_batch_excluded(self._h)

    def resource(self, review: int):
        """HandleViolation's Resource identity (target.go:193-244):
        (apiVersion, kind, name, namespace) of the review's object"""
        r = _Resource()
        rc = self._drv._lib.gk_batch_resource(self._drv._e, self._h, review, C.byref(r))
        if rc not in (0, 6):
            self._drv._check(rc)
        dec = lambda b: b.decode("utf-8", "surrogateescape")  # noqa: E731
        return dec(r.api_version), dec(r.kind), dec(r.name), dec(r.namespace)

    def stats(self):
        """(reviews, document nodes, distinct string-value bytes, match-column bytes)."""
        v = [C.c_uint64() for _ in range(4)]
        self._drv._lib.gk_batch_stats(self._h, *[C.byref(x) for x in v])
        return tuple(x.value for x in v)

    def free(self):
        if self._h:
            self._drv._lib.gk_batch_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Driver:
    """drivers.Driver over libgkgpu (interface.go:21-39)."""

    def __init__(self, device: int = 0, jit: bool = True, host_only: bool = False, coalesce_us: int = 0,
                 coalesce_max: int = 256):
        """jit=False pins every template to the bytecode VM kernel (A/B parity);
        host_only=True stages batches on the host only (CPU baseline, tests);
        coalesce_us > 0 gathers concurrent query(violation) calls into one
        launch of up to coalesce_max reviews (the webhook micro-batch
        coalescer, include/gkgpu.h)."""
        self._lib = load_library()
        e = C.c_void_p()
        opts = {"device": device, "jit": jit}
        if host_only:
            opts["host_only"] = True
        if coalesce_us:
            opts["coalesce_us"] = int(coalesce_us)
            opts["coalesce_max"] = int(coalesce_max)
        rc = self._lib.gk_engine_create(_b(json.dumps(opts)), C.byref(e))
        if rc != 0:
            raise EngineUnavailable("gk_engine_create failed (%d)" % rc)
        self._e = e

    def close(self):
        if self._e:
            self._lib.gk_engine_destroy(self._e)
            self._e = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            msg = self._lib.gk_last_error(self._e).decode("utf-8", "replace")
            if rc == 4:
                raise EngineUnavailable(msg)
            if rc == 3:
                raise QueryError(msg)
            raise RuntimeError("gkgpu error %d: %s" % (rc, msg))

    @staticmethod
    def device_available() -> bool:
        return bool(load_library().gk_device_available())

    # -- Driver.Init (interface.go:22)
    def init(self):
        self._check(self._lib.gk_init(self._e))

    # -- Driver.PutModule (interface.go:24)
    def put_module(self, name: str, src: str):
        s = _b(src)
        self._check(self._lib.gk_put_module(self._e, _b(name), s, len(s)))

    # -- Driver.PutModules (interface.go:26)
    def put_modules(self, prefix: str, srcs: Sequence[str]):
        arr, lens, _keep = _arr(srcs)
        self._check(self._lib.gk_put_modules(self._e, _b(prefix), arr, lens, len(srcs)))

    # -- Driver.DeleteModule (interface.go:28)
    def delete_module(self, name: str) -> bool:
        d = C.c_int()
        self._check(self._lib.gk_delete_module(self._e, _b(name), C.byref(d)))
        return bool(d.value)

    # -- Driver.DeleteModules (interface.go:30)
    def delete_modules(self, prefix: str) -> int:
        d = C.c_int()
        self._check(self._lib.gk_delete_modules(self._e, _b(prefix), C.byref(d)))
        return d.value

    # -- Driver.PutData (interface.go:32)
    def put_data(self, path: str, data):
        js = _b(data if isinstance(data, str) else json.dumps(data))
        self._check(self._lib.gk_put_data(self._e, _b(path), js, len(js)))

    # -- Driver.DeleteData (interface.go:34)
    def delete_data(self, path: str) -> bool:
        d = C.c_int()
        self._check(self._lib.gk_delete_data(self._e, _b(path), C.byref(d)))
        return bool(d.value)

    # -- Driver.Query (interface.go:36)
    def query(self, path: str, input_val=None) -> Results:
        js = _b(input_val if isinstance(input_val, str) else json.dumps(input_val))
        out = C.c_void_p()
        self._check(self._lib.gk_query(self._e, _b(path), js, len(js), C.byref(out)))
        return _collect(self._lib, out)

    def audit_cache_stats(self):
        """(builds, reviews) of the device-resident from-cache batch hooks.audit
        evaluates (gk_audit_cache_stats): a build per engine state"""
        b, r = C.c_uint64(), C.c_uint64()
        self._lib.gk_audit_cache_stats.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        self._check(self._lib.gk_audit_cache_stats(self._e, C.byref(b), C.byref(r)))
        return b.value, r.value

    def audit_sample(self, limit: int = 20) -> AuditSweep:
        """--audit-from-cache as the audit manager consumes it
        (gk_audit_cache_sample): Client.Audit over the synced inventory's
        staged batch, reduced on the device to exact per-constraint totals and
        the first `limit` results per constraint (manager.go:195-207,
        :462-508); review indexes are inventory path order"""
        out = C.c_void_p()
        self._lib.gk_audit_cache_sample.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_void_p)]
        self._check(self._lib.gk_audit_cache_sample(self._e, limit, C.byref(out)))
        return _collect_audit(self._lib, out)

    def audit_summary(self):
        """Client.Audit (hooks.audit) without materializing Python rows: the
        per-constraint totals, the result count and the engine phase timings"""
        out = C.c_void_p()
        self._check(self._lib.gk_query(self._e, _b('hooks["%s"].audit' % TARGET), b"null", 4, C.byref(out)))
        try:
            n = self._lib.gk_results_count(out)
            nc = self._lib.gk_results_constraints(out)
            totals = [self._lib.gk_results_constraint_total(out, i) for i in range(nc)]
            ms = (C.c_double * 5)()
            self._lib.gk_results_timing(out, ms)
            return {"results": n, "totals": totals, "timing_ms": list(ms),
                    "launches": [(k.kernel, round(k.ms, 3), k.tuples) for k in _launches(self._lib, out)]}
        finally:
            self._lib.gk_results_free(out)

    def coalesce_stats(self):
        """(launches, gk_query calls served) of the micro-batch coalescer"""
        b, r = C.c_uint64(), C.c_uint64()
        self._check(self._lib.gk_coalesce_stats(self._e, C.byref(b), C.byref(r)))
        return b.value, r.value

    # -- Driver.Dump (interface.go:38)
    def dump(self) -> str:
        p = C.c_void_p()
        self._check(self._lib.gk_dump(self._e, C.byref(p)))
        s = C.string_at(p).decode()
        self._lib.gk_free_string(p)
        return s

    # -- batch extensions
    def query_batch(self, inputs: Sequence) -> Results:
        strs = [x if isinstance(x, str) else json.dumps(x) for x in inputs]
        arr, lens, _keep = _arr(strs)
        out = C.c_void_p()
        self._check(self._lib.gk_query_batch(self._e, arr, lens, len(strs), C.byref(out)))
        return _collect(self._lib, out)

    def query_batch_export(self, inputs: Sequence):
        """gk_query_batch, then every result row copied out in one call
        (gk_results_export) -- what a native caller does with the result views
        -- plus the per-review status words.  Returns (blob, status); parse
        the rows with export_rows(blob)."""
        strs = [x if isinstance(x, str) else json.dumps(x) for x in inputs]
        arr, lens, _keep = _arr(strs)
        out = C.c_void_p()
        self._check(self._lib.gk_query_batch(self._e, arr, lens, len(strs), C.byref(out)))
        h = out
        try:
            need = C.c_size_t()
            self._lib.gk_results_export(h, None, 0, C.byref(need))
            buf = C.create_string_buffer(max(1, need.value))
            self._check(self._lib.gk_results_export(h, buf, need.value, C.byref(need)))
            nr = self._lib.gk_results_reviews(h)
            st = (C.c_uint32 * max(1, nr))()
            self._lib.gk_results_copy_status(h, st, None)
            return buf.raw[:need.value], st[:nr]
        finally:
            self._lib.gk_results_free(h)

    def query_export(self, path: str, input_json):
        """Driver.Query of one input (bytes / str JSON), its rows copied out in
        one gk_results_export call: (blob, status word).  With the coalescer
        on, concurrent calls share launches."""
        js = input_json if isinstance(input_json, bytes) else _b(input_json)
        out = C.c_void_p()
        self._check(self._lib.gk_query(self._e, _b(path), js, len(js), C.byref(out)))
        h = out
        try:
            need = C.c_size_t()
            self._lib.gk_results_export(h, None, 0, C.byref(need))
            buf = C.create_string_buffer(max(1, need.value))
            self._check(self._lib.gk_results_export(h, buf, need.value, C.byref(need)))
            st = (C.c_uint32 * 1)()
            self._lib.gk_results_copy_status(h, st, None)
            return buf.raw[:need.value], st[0]
        finally:
            self._lib.gk_results_free(h)

    def review_objects(self, objs: Sequence, namespaces: Sequence) -> Results:
        o = [x if isinstance(x, str) else json.dumps(x) for x in objs]
        n = [None if x is None else (x if isinstance(x, str) else json.dumps(x)) for x in namespaces]
        oa, ol, _k1 = _arr(o)
        na, nl, _k2 = _arr(n)
        out = C.c_void_p()
        self._check(self._lib.gk_review_objects(self._e, oa, ol, na, nl, len(o), C.byref(out)))
        return _collect(self._lib, out)

    @staticmethod
    def _page_args(page):
        import numpy as np
        oo = np.ascontiguousarray(page.obj_offs, dtype=np.uint64)
        no = np.ascontiguousarray(page.ns_offs, dtype=np.uint64)
        on = np.ascontiguousarray(page.obj_ns, dtype=np.uint32)
        keep = (oo, no, on)
        return [page.objs, oo.ctypes.data, page.n, page.nss, no.ctypes.data, page.n_ns, on.ctypes.data], keep

    def review_page(self, page) -> Results:
        """audit discovery mode over one List page (gkgpu.page.Page)"""
        args, _keep = self._page_args(page)
        out = C.c_void_p()
        self._check(self._lib.gk_review_page(self._e, *args, C.byref(out)))
        return _collect(self._lib, out)

    def stage_page(self, page) -> Batch:
        """stage one List page (gkgpu.page.Page) on the device"""
        args, _keep = self._page_args(page)
        out = C.c_void_p()
        self._check(self._lib.gk_batch_stage_page(self._e, *args, C.byref(out)))
        return Batch(self, out, page.n)

    def debug_flatten(self, page, threads: int = 0):
        """flatten a page on the host only: (content hash, nodes, parse ms, total ms)"""
        args, _keep = self._page_args(page)
        h, n = C.c_uint64(), C.c_uint64()
        ms = (C.c_double * 2)()
        self._check(self._lib.gk_debug_flatten_page(self._e, *args, threads, C.byref(h), C.byref(n), ms))
        return h.value, n.value, ms[0], ms[1]

    def debug_batch_hash(self, batch) -> int:
        """content hash of a staged batch as the kernels see it (its device node
        array and review columns downloaded; equal to debug_flatten's hash of
        the same page)"""
        h = C.c_uint64()
        self._lib.gk_debug_batch_hash.argtypes = [C.c_void_p, C.c_void_p, C.POINTER(C.c_uint64)]
        self._check(self._lib.gk_debug_batch_hash(self._e, batch._h, C.byref(h)))
        return h.value

    # -- process excluder (excluder.go)
    def excluder_add(self, processes: Sequence[str], namespaces: Sequence[str]):
        """Excluder.Add(MatchEntry{ExcludedNamespaces, Processes}) (excluder.go:44-68)"""
        pa, _, _k1 = _arr(list(processes))
        na, _, _k2 = _arr(list(namespaces))
        self._check(self._lib.gk_excluder_add(self._e, pa, len(processes), na, len(namespaces)))

    def excluder_clear(self):
        self._check(self._lib.gk_excluder_clear(self._e))

    def is_namespace_excluded(self, process: str, namespace: str) -> bool:
        """Excluder.IsNamespaceExcluded (excluder.go:82-86)"""
        return bool(self._lib.gk_excluder_is_excluded(self._e, _b(process), _b(namespace)))

    def debug_stage_cache(self) -> Batch:
        """a staged batch of hooks.audit's from-cache reviews of the synced
        inventory, in inventory path order (tests: the CPU checker)"""
        out = C.c_void_p()
        self._lib.gk_debug_stage_cache.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
        self._check(self._lib.gk_debug_stage_cache(self._e, C.byref(out)))
        n = C.c_uint64()
        self._lib.gk_batch_stats(out, C.byref(n), None, None, None)
        return Batch(self, out, n.value)

    def debug_stage_inputs(self, inputs: Sequence) -> Batch:
        """a staged batch of Query inputs ({"review": ...}; diagnostics / tests)"""
        strs = [x if isinstance(x, str) else json.dumps(x) for x in inputs]
        arr, lens, _keep = _arr(strs)
        out = C.c_void_p()
        self._lib.gk_debug_stage_inputs.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                                                    C.c_size_t, C.POINTER(C.c_void_p)]
        self._check(self._lib.gk_debug_stage_inputs(self._e, arr, lens, len(strs), C.byref(out)))
        return Batch(self, out, len(strs))

    def stage_objects(self, objs: Sequence, namespaces: Sequence) -> Batch:
        o = [x if isinstance(x, str) else json.dumps(x) for x in objs]
        n = [None if x is None else (x if isinstance(x, str) else json.dumps(x)) for x in namespaces]
        oa, ol, _k1 = _arr(o)
        na, nl, _k2 = _arr(n)
        out = C.c_void_p()
        self._check(self._lib.gk_batch_stage_objects(self._e, oa, ol, na, nl, len(o), C.byref(out)))
        return Batch(self, out, len(o))

    # -- introspection
    def debug_store_sizes(self):
        """(nodes of the permanent region, interned strings) as the next evaluation sees them"""
        n, st = C.c_uint64(), C.c_uint64()
        self._lib.gk_debug_store_sizes.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        self._check(self._lib.gk_debug_store_sizes(self._e, C.byref(n), C.byref(st)))
        return n.value, st.value

    def debug_clock_mhz(self) -> float:
        """the shader clock (MHz) a spinning wavefront measures on this device
        (s_memtime over the 100 MHz s_memrealtime reference)"""
        v = C.c_double()
        self._lib.gk_debug_clock_mhz.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
        self._check(self._lib.gk_debug_clock_mhz(self._e, C.byref(v)))
        return v.value

    def debug_disasm(self, kind: str) -> str:
        """bytecode listing of a compiled template (diagnostics; with GKGPU_PROFILE=2
        the first column is the last launch's per-instruction execution count)"""
        p = C.c_void_p()
        self._lib.gk_debug_disasm.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_void_p)]
        self._check(self._lib.gk_debug_disasm(self._e, _b(kind), C.byref(p)))
        s = C.string_at(p).decode()
        self._lib.gk_free_string(p)
        return s

    def prepare(self, device: bool = True):
        """gk_engine_prepare: compile and upload the current templates and
        constraints now (the reference compiles at AddTemplate), so the next
        staging / evaluation does not"""
        self._lib.gk_engine_prepare.argtypes = [C.c_void_p, C.c_int]
        self._check(self._lib.gk_engine_prepare(self._e, 1 if device else 0))

    def template_backend(self, kind: str):
        """(backend, detail): 2 template kernel (hipRTC), 1 bytecode VM, 3 guard program on
        the GPU + CPU fallback for the reviews that reach an unsupported expression,
        0 CPU fallback for every matched review"""
        b, d = C.c_int(), C.c_char_p()
        self._check(self._lib.gk_template_backend(self._e, _b(kind), C.byref(b), C.byref(d)))
        return b.value, (d.value or b"").decode("utf-8", "replace")

    def template_joins(self, kind: str):
        """the template's inventory join sites (compiler.cc join_site): a list of
        data.inventory paths whose iteration probes a per-constraint hash index"""
        d = C.c_char_p()
        n = self._lib.gk_template_joins(self._e, _b(kind), C.byref(d))
        if n < 0:
            self._check(n)
        s = (d.value or b"").decode("utf-8", "replace")
        return s.split(";") if n else []

    def join_stats(self) -> dict:
        """the join indexes of the current state (built on the device when the
        engine is prepared): indexes, entries, unindexed sites, leaves, build ms"""
        v = [C.c_uint64() for _ in range(4)]
        ms = C.c_double()
        self._check(self._lib.gk_join_stats(self._e, *[C.byref(x) for x in v], C.byref(ms)))
        return {"indexes": v[0].value, "entries": v[1].value, "unindexed": v[2].value, "leaves": v[3].value,
                "build_ms": ms.value}

    def template_status(self, kind: str):
        r = C.c_char_p()
        st = self._lib.gk_template_status(self._e, _b(kind), C.byref(r))
        return st, (r.value.decode() if r.value else "")

    def constraints(self):
        n = self._lib.gk_constraint_count(self._e)
        out = []
        for i in range(n):
            k, nm = C.c_char_p(), C.c_char_p()
            self._lib.gk_constraint_info(self._e, i, C.byref(k), C.byref(nm))
            out.append((k.value.decode(), nm.value.decode()))
        return out


def export_rows(blob: bytes):
    """(review, constraint index, msg, details JSON) of every row of a
    gk_results_export buffer, in result order."""
    import struct
    out = []
    i, n = 0, len(blob)
    while i < n:
        rv, c, ml, dl = struct.unpack_from("<IIII", blob, i)
        i += 16
        msg = blob[i:i + ml].decode("utf-8", "surrogateescape")
        i += ml
        det = blob[i:i + dl].decode("utf-8", "surrogateescape")
        i += dl
        out.append((rv, c, msg, det))
    return out
