"""GPU probe: cost breakdown of the K8sContainerLimits predicate by template variants."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402

COMPILE_ONLY = "--compile-only" in sys.argv
argv = [a for a in sys.argv[1:] if a != "--compile-only"]
N = int(argv[0]) if argv else 1_000_000
ts, cs = W.config2()
cl_t = [t for t in ts if t["spec"]["crd"]["spec"]["names"]["kind"] == "K8sContainerLimits"][0]
cl_c = [c for c in cs if c["kind"] == "K8sContainerLimits"][0]
src = cl_t["spec"]["targets"][0]["rego"]
head, gv = src.split("violation[{\"msg\": msg}] {", 1)
helpers = head
bodies = re.findall(r"general_violation\[\{\"msg\": msg, \"field\": field\}\] \{(.*?)\n\}", src, re.S)

GV = 'general_violation[{"msg": msg, "field": field}] {%s\n}\n'
VIOL = ('violation[{"msg": msg}] {\n\tgeneral_violation[{"msg": msg, "field": "containers"}]\n}\n\n'
        'violation[{"msg": msg}] {\n\tgeneral_violation[{"msg": msg, "field": "initContainers"}]\n}\n\n')


def const_msg(b):
    return re.sub(r"msg := sprintf\(.*\)", 'msg := "x"', b)


variants = {
    "full": helpers + VIOL + "".join(GV % b for b in bodies),
    "iter_only": helpers + VIOL + GV % '\n\tcontainer := input.review.object.spec[field][_]\n\tcontainer.name == "zz-never"\n\tmsg := "x"',
    "gets_only": helpers + VIOL + "".join(
        GV % ('\n\tcontainer := input.review.object.spec[field][_]\n\tx := container.resources.limits.%s\n\tx == "zz-never"\n\tmsg := "x"' % f)
        for f in ("cpu", "memory")),
    "bodies_3to6": helpers + VIOL + "".join(GV % b for b in bodies[2:6]),
    "canon_no_msgs": helpers + VIOL + "".join(GV % const_msg(b) for b in (bodies[0], bodies[1], bodies[6], bodies[7])),
    "full_const_msg": helpers + VIOL + "".join(GV % const_msg(b) for b in bodies),
    "canon_cpu_only": helpers + VIOL + "".join(GV % const_msg(b) for b in (bodies[0], bodies[6])),
    "canon_mem_only": helpers + VIOL + "".join(GV % const_msg(b) for b in (bodies[1], bodies[7])),
}
objs, nss = W.gen_pods_json(N, seed=42, n_namespaces=1000)
for name, rego in variants.items():
    t = dict(cl_t)
    t["spec"] = dict(cl_t["spec"])
    t["spec"]["targets"] = [dict(cl_t["spec"]["targets"][0], rego=rego)]
    d = gkgpu.Driver()
    cl = Client(d)
    cl.add_template(t)
    cl.add_constraint(cl_c)
    be = d.template_backend("K8sContainerLimits")
    if COMPILE_ONLY:
        print(name, be, flush=True)
        continue
    b = d.stage_objects(objs, nss)
    b.eval(decode=False, light=True)
    r = b.eval(decode=False, light=True)
    print("%-16s backend %d kernel %.2f ms tuples %d bytes %d" % (name, be[0], r.timing_ms[2], r.device_tuples,
                                                                 r.device_bytes), flush=True)
    b.free()
    d.close()
