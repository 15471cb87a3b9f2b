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
    # every lookup is either still a call or a copy
    assert on.count("= vget(L,") == off.count("= vget(L,")


def test_lazy_sprintf_argument_count_is_an_immediate():
    src = _dump("K8sRequiredProbes")
    assert "lazy_sprintf_n(L," in src
    assert "lazy_sprintf(L," not in src
