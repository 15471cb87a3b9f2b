"""Template-kernel source generation (jit.cc), checked on the host: no GPU
needed to generate the HIP source (GKGPU_JIT_DUMP keeps it; hipRTC compiles it
on the device box).  The GPU parity suite runs the same kernels."""
import glob
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dump(kind, env_extra=()):
    d = tempfile.mkdtemp(prefix="gkjit_test")
    code = r'''
import sys
sys.path[:0] = [%r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client
ts, cs = W.config2()
d = gkgpu.Driver()
cl = Client(d)
for t in ts:
    if t["spec"]["crd"]["spec"]["names"]["kind"] == %r:
        cl.add_template(t)
print(d.template_backend(%r))
''' % (ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), kind, kind)
    env = dict(os.environ, GKGPU_JIT_CACHE="0", GKGPU_JIT_DUMP=d, GKGPU_JIT_DUMP_ONLY="1", **dict(env_extra))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    files = glob.glob(os.path.join(d, "*.hip"))
    assert len(files) == 1, files
    return open(files[0]).read()


def test_lookup_cse_reuses_prologue_lookups_in_inlined_calls():
    """K8sContainerLimits: missing(container.resources.limits, "cpu") reads the
    value the fused group's prologue looked up; the generated code copies the
    register instead of scanning the object again (jit.cc look_flow)."""
    on = _dump("K8sContainerLimits")
    off = _dump("K8sContainerLimits", [("GKGPU_JIT_CSE", "0")])
    reused = on.count("// = vget(")
    assert reused >= 8, reused
    assert off.count("// = vget(") == 0
    # every lookup is either still a call, a copy, or already in its register
    calls = lambda src: src.count("= vget(L,") + src.count("= vget_p(L,")  # noqa: E731
    assert calls(on) + on.count(" holds ") == calls(off) + off.count(" holds ")


def test_computed_key_lookup_reuses_its_shadow():
    """jit.cc look_flow computed-key facts: K8sRequiredProbes reads
    ctr[probe] in probe_is_missing's first body and again in
    probe_field_empty; the second read copies the first's shadow local (the
    result register itself is reused in between).  GKGPU_JIT_DYNCSE=0: both
    scan the container."""
    on = _dump("K8sRequiredProbes")
    off = _dump("K8sRequiredProbes", [("GKGPU_JIT_DYNCSE", "0")])
    import re
    assert re.search(r"uint64_t dk\d+ = 0;", on)
    assert re.search(r"= dk\d+;  // = vget\(L, ", on)
    assert "dk" not in off.split("_pred(")[1]


def test_parameter_reads_come_from_the_wave_lds_stage():
    """jit.cc param_flow: lookups and iterations over the constraint's
    parameters read the wave's LDS copy of the subtree (devrt.h stage_wave,
    vget_p / op_iter_next_p) when the kernel's LDS budget has room; a
    re_match with a computed pattern also stages the compressed DFAs
    (GK_LDS_DFA).  GKGPU_LDS_STAGE=0 turns both off.  K8sContainerLimits
    probes the memo at more sites than it reads parameters, so its budget goes
    to the memo cache first (GK_LDS_MEMO, jit.cc stage_plan); without the cache
    the parameters take the room."""
    assert "#define GK_LDS_MEMO 32" in _dump("K8sContainerLimits")
    lim = _dump("K8sContainerLimits", [("GKGPU_JIT_LDSMEMO", "0")])
    assert "#define GK_LDS_PARAMS 1" in lim and "GK_LDS_MEMO" not in lim
    assert "= vget_p(L, " in lim
    assert "#define GK_LDS_DFA 1" not in lim  # no computed re_match pattern
    lab = _dump("K8sRequiredLabels")
    assert "#define GK_LDS_DFA 1" in lab and "#define GK_LDS_PARAMS 1" in lab
    assert "!op_iter_next_p(L, " in lab
    off = _dump("K8sRequiredLabels", [("GKGPU_LDS_STAGE", "0")])
    assert "GK_LDS_PARAMS" not in off and "GK_LDS_DFA" not in off
    assert "= vget_p(L, " not in off and "!op_iter_next_p(L, " not in off


def test_lazy_sprintf_argument_count_is_an_immediate():
    # (with the list built: the fused emission otherwise drops it, below)
    src = _dump("K8sRequiredProbes", [("GKGPU_JIT_EMITDCE", "0")])
    assert "lazy_sprintf_n(L," in src
    assert "lazy_sprintf(L," not in src


def test_required_probes_builds_no_sets_after_the_rewrite():
    """rego.cc optimize_sets: probe_field_empty's two sets and their difference
    are gone from K8sRequiredProbes' kernel (GKGPU_REGO_SETS=0 keeps them)."""
    assert "arith(L, 1u," not in _dump("K8sRequiredProbes")
    assert "arith(L, 1u," in _dump("K8sRequiredProbes", [("GKGPU_REGO_SETS", "0")])


def test_required_labels_builds_no_provided_set():
    """rego.cc optimize_sets (second pattern): k8srequiredlabels' `provided`
    set is not built; `missing` iterates `required` with a lookup per key"""
    on, off = _dump("K8sRequiredLabels"), _dump("K8sRequiredLabels", [("GKGPU_REGO_SETS", "0")])
    assert "arith(L, 1u," not in on and "arith(L, 1u," in off


def test_fused_emission_builds_no_argument_list():
    """jit.cc dce_sites: K8sContainerLimits' violation messages are sprintfs
    whose argument lists exist only for the emission; the fused emission takes
    the arguments from the shadow copies and the list is not built
    (op_emit_args_build rebuilds it only on the slow path).
    GKGPU_JIT_EMITDCE=0 keeps the lists."""
    on = _dump("K8sContainerLimits")
    off = _dump("K8sContainerLimits", [("GKGPU_JIT_EMITDCE", "0")])
    assert "op_emit_args_build(L," in on
    assert "list_new(L," not in on
    assert "op_emit_args_build(L," not in off
    assert "list_new(L," in off and "op_emit_args(L," in off


def test_yield_into_an_undefined_output_is_a_copy():
    """jit.cc: a yield whose output register holds undefined on every path
    (EmitFlow.undef_at) is a plain copy -- no conflict check, so a deferred
    sprintf passes through it unforced and K8sRequiredProbes' message list is
    dropped too (jit.cc dce_sites)."""
    src = _dump("K8sRequiredProbes")
    assert "op_emit_args_build(L," in src
    assert "list_new(L, 2u" not in src


def _dump_c3(kind, env_extra=()):
    d = tempfile.mkdtemp(prefix="gkjit_test")
    code = r'''
import sys
sys.path[:0] = [%r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client
ts, cs = W.config3()
d = gkgpu.Driver()
cl = Client(d)
for t in ts:
    if t["spec"]["crd"]["spec"]["names"]["kind"] == %r:
        cl.add_template(t)
print(d.template_backend(%r))
''' % (ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), kind, kind)
    env = dict(os.environ, GKGPU_JIT_CACHE="0", GKGPU_JIT_DUMP=d, GKGPU_JIT_DUMP_ONLY="1", **dict(env_extra))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    files = glob.glob(os.path.join(d, "*.hip"))
    assert len(files) == 1, files
    return open(files[0]).read()


def test_details_object_of_a_fused_emission_is_not_built():
    """jit.cc kv_sites: k8sallowedlabelregex's {"label": key} details object
    is built right before its emission and read nowhere else; the emission
    takes the key and value registers (devrt.h op_emit_args_kvd) and builds
    the object only on its slow path.  GKGPU_JIT_KVDCE=0 keeps it."""
    on = _dump_c3("K8sAllowedLabelRegex")
    off = _dump_c3("K8sAllowedLabelRegex", [("GKGPU_JIT_KVDCE", "0")])
    assert "op_emit_args_kvd<true>(L," in on and "op_obj_put(L," not in on.split("_pred(")[1]
    assert "op_emit_args_kvd" not in off.split("_pred(")[1] and "op_obj_put(L," in off


ALIASED_LIST = r'''package k8saliasedlist

violation[{"msg": msg}] {
	name := input.review.object.metadata.name
	args := [name, "x"]
	outer := [args]
	msg := sprintf("%v is %v", args)
	outer[0][0] == name
}
'''
PLAIN_LIST = r'''package k8splainlist

violation[{"msg": msg}] {
	name := input.review.object.metadata.name
	msg := sprintf("%v is %v", [name, "x"])
}
'''


def _dump_rego(kind, rego):
    d = tempfile.mkdtemp(prefix="gkjit_test")
    code = r'''
import sys
sys.path[:0] = [%r, %r]
import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client
d = gkgpu.Driver()
cl = Client(d)
cl.add_template(W._tmpl(%r, %r))
print(d.template_backend(%r))
''' % (ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), kind, rego, kind)
    env = dict(os.environ, GKGPU_JIT_CACHE="0", GKGPU_JIT_DUMP=d, GKGPU_JIT_DUMP_ONLY="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    files = glob.glob(os.path.join(d, "*.hip"))
    assert len(files) == 1, files
    return open(files[0]).read()


def test_argument_list_read_elsewhere_is_still_built():
    """ADVICE r05 (jit.cc dce_sites): an emission-only sprintf argument list is
    not built (its fused emission has the arguments) -- but only when nothing
    between its LIST_NEW and the sprintf reads it except its own LIST_ADDs.
    Here the list is also added into `outer`, which the body reads, so it must
    be built; the plain form still drops it."""
    marker = "the argument list of a fused emission"
    assert marker in _dump_rego("K8sPlainList", PLAIN_LIST)
    assert marker not in _dump_rego("K8sAliasedList", ALIASED_LIST)
