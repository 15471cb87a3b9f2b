"""GPU probe: cost breakdown of the K8sRequiredProbes predicate by template
variants (config 2, 1M Pods): kernel time of each variant of the template."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gatekeeper-1_amd"), os.path.join(ROOT, "tests")]
import gkgpu  # noqa: E402
from gkgpu import workloads as W  # noqa: E402
from gkgpu.client import Client  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
ts, cs = W.config2()
rp_t = [t for t in ts if t["spec"]["crd"]["spec"]["names"]["kind"] == "K8sRequiredProbes"][0]
rp_c = [c for c in cs if c["kind"] == "K8sRequiredProbes"][0]
src = rp_t["spec"]["targets"][0]["rego"]

HEAD = src[:src.index("violation[")]
VIOL = src[src.index("violation["):src.index("probe_is_missing(ctr, probe) = true {")]
MISSING1 = 'probe_is_missing(ctr, probe) = true {\n\tnot ctr[probe]\n}\n\n'
MISSING2 = 'probe_is_missing(ctr, probe) = true {\n\tprobe_field_empty(ctr, probe)\n}\n\n'
REST = src[src.index("probe_field_empty(ctr, probe) = true {"):]
CONST_MSG = VIOL.replace("msg := get_violation_message(container, input.review, probe)", 'msg := "x"')
EMPTY_ALT = ('probe_field_empty(ctr, probe) = true {\n\tcount(ctr[probe]) == 0\n}\n\n' +
             REST[REST.index("get_violation_message"):])

INLINE_MSG = VIOL.replace("msg := get_violation_message(container, input.review, probe)",
                          'msg := sprintf("Container <%v> in your <%v> <%v> has no <%v>", '
                          '[container.name, input.review.kind.kind, input.review.object.metadata.name, probe])')
ONE_ARG = VIOL.replace("msg := get_violation_message(container, input.review, probe)",
                       'msg := sprintf("Container <%v> has no probe", [container.name])')
CONST_ARGS = VIOL.replace("msg := get_violation_message(container, input.review, probe)",
                          'msg := sprintf("Container <%v> in your <%v> <%v> has no <%v>", ["a", "b", "c", "d"])')
only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
variants = {
    "full": src,
    "const_msg": HEAD + CONST_MSG + MISSING1 + MISSING2 + REST,
    "missing_only": HEAD + VIOL + MISSING1 + REST,
    "missing_only_const_msg": HEAD + CONST_MSG + MISSING1 + REST,
    "empty_by_count": HEAD + VIOL + MISSING1 + MISSING2 + EMPTY_ALT,
    "inline_msg": HEAD + INLINE_MSG + MISSING1 + MISSING2 + REST,
    "one_arg_msg": HEAD + ONE_ARG + MISSING1 + MISSING2 + REST,
    "const_args_msg": HEAD + CONST_ARGS + MISSING1 + MISSING2 + REST,
    "loops_only": HEAD + ('violation[{"msg": msg}] {\n\tcontainer := input.review.object.spec.containers[_]\n'
                          '\tprobe := input.parameters.probes[_]\n\tcontainer.name == "zz-never"\n\tmsg := "x"\n}\n'),
}
objs, nss = W.gen_pods_json(N, seed=42, n_namespaces=1000)
for name, rego in variants.items():
    if only and name not in only:
        continue
    t = dict(rp_t)
    t["spec"] = dict(rp_t["spec"])
    t["spec"]["targets"] = [dict(rp_t["spec"]["targets"][0], rego=rego)]
    d = gkgpu.Driver()
    cl = Client(d)
    cl.add_template(t)
    cl.add_constraint(rp_c)
    be = d.template_backend("K8sRequiredProbes")
    b = d.stage_objects(objs, nss)
    b.eval(decode=False, light=True)
    r = b.eval(decode=False, light=True)
    ks = [(k, round(ms, 2)) for k, ms, _n in r.launches]
    print("%-24s backend %d %s tuples %d" % (name, be[0], ks, r.device_tuples), flush=True)
