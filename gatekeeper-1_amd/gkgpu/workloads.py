"""BASELINE workloads: ConstraintTemplates, Constraints and seeded synthetic resources.

Templates are the demo policies BASELINE.json names, written out here in the
form the driver receives them (OPA-formatted module text; client.go:332-339
re-prints sources with format.Ast), so tests and the bench run where the
reference tree is absent:

* K8sRequiredLabels (basic)   — demo/basic/templates/k8srequiredlabels_template.yaml
* K8sRequiredLabels (regex)   — demo/agilebank/templates/k8srequiredlabels_template.yaml
* K8sAllowedRepos             — demo/agilebank/templates/k8sallowedrepos_template.yaml
* K8sContainerLimits          — demo/agilebank/templates/k8scontainterlimits_template.yaml
* K8sRequiredProbes           — demo/agilebank/templates/k8srequiredprobes_template.yaml
* K8sAllowedLabelRegex / K8sAllowedAnnotationRegex — build-authored allowedRegex
  variants for config 3, same Rego subset.

Generators follow SURVEY 8(d)'s synthetic-input spec with the seeds given there.
"""
from __future__ import annotations

import json
import random

TARGET = "admission.k8s.gatekeeper.sh"


def _tmpl(kind, rego, schema=None):
    return {
        "apiVersion": "templates.gatekeeper.sh/v1beta1",
        "kind": "ConstraintTemplate",
        "metadata": {"name": kind.lower()},
        "spec": {"crd": {"spec": {"names": {"kind": kind}, "validation": {"openAPIV3Schema": schema or {}}}},
                 "targets": [{"target": TARGET, "rego": rego}]},
    }


REQUIRED_LABELS_BASIC = _tmpl("K8sRequiredLabels", """package k8srequiredlabels

violation[{"msg": msg, "details": {"missing_labels": missing}}] {
	provided := {label | input.review.object.metadata.labels[label]}
	required := {label | label := input.parameters.labels[_]}
	missing := required - provided
	count(missing) > 0
	msg := sprintf("you must provide labels: %v", [missing])
}
""")

REQUIRED_LABELS = _tmpl("K8sRequiredLabels", """package k8srequiredlabels

get_message(parameters, _default) = msg {
	not parameters.message
	msg := _default
}

get_message(parameters, _default) = msg {
	msg := parameters.message
}

violation[{"msg": msg, "details": {"missing_labels": missing}}] {
	provided := {label | input.review.object.metadata.labels[label]}
	required := {label | label := input.parameters.labels[_].key}
	missing := required - provided
	count(missing) > 0
	def_msg := sprintf("you must provide labels: %v", [missing])
	msg := get_message(input.parameters, def_msg)
}

violation[{"msg": msg}] {
	value := input.review.object.metadata.labels[key]
	expected := input.parameters.labels[_]
	expected.key == key

	# do not match if allowedRegex is not defined, or is an empty string
	expected.allowedRegex != ""
	not re_match(expected.allowedRegex, value)
	def_msg := sprintf("Label <%v: %v> does not satisfy allowed regex: %v", [key, value, expected.allowedRegex])
	msg := get_message(input.parameters, def_msg)
}
""")

ALLOWED_REPOS = _tmpl("K8sAllowedRepos", """package k8sallowedrepos

violation[{"msg": msg}] {
	container := input.review.object.spec.containers[_]
	satisfied := [good | repo = input.parameters.repos[_]; good = startswith(container.image, repo)]
	not any(satisfied)
	msg := sprintf("container <%v> has an invalid image repo <%v>, allowed repos are %v", [container.name, container.image, input.parameters.repos])
}

violation[{"msg": msg}] {
	container := input.review.object.spec.initContainers[_]
	satisfied := [good | repo = input.parameters.repos[_]; good = startswith(container.image, repo)]
	not any(satisfied)
	msg := sprintf("container <%v> has an invalid image repo <%v>, allowed repos are %v", [container.name, container.image, input.parameters.repos])
}
""")

_MEM = [("E", "1000000000000000000000"), ("P", "1000000000000000000"), ("T", "1000000000000000"),
        ("G", "1000000000000"), ("M", "1000000000"), ("k", "1000000"), ("", "1000"), ("m", "1"),
        ("Ki", "1024000"), ("Mi", "1048576000"), ("Gi", "1073741824000"), ("Ti", "1099511627776000"),
        ("Pi", "1125899906842624000"), ("Ei", "1152921504606846976000")]

CONTAINER_LIMITS = _tmpl("K8sContainerLimits", """package k8scontainerlimits

missing(obj, field) = true {
	not obj[field]
}

missing(obj, field) = true {
	obj[field] == ""
}

canonify_cpu(orig) = new {
	is_number(orig)
	new := orig * 1000
}

canonify_cpu(orig) = new {
	not is_number(orig)
	endswith(orig, "m")
	new := to_number(replace(orig, "m", ""))
}

canonify_cpu(orig) = new {
	not is_number(orig)
	not endswith(orig, "m")
	re_match("^[0-9]+$", orig)
	new := to_number(orig) * 1000
}
""" + "".join('\nmem_multiple("%s") = %s {\n\ttrue\n}\n' % (s, v) for s, v in _MEM) + """
get_suffix(mem) = suffix {
	not is_string(mem)
	suffix := ""
}

get_suffix(mem) = suffix {
	is_string(mem)
	count(mem) > 0
	suffix := substring(mem, count(mem) - 1, -1)
	mem_multiple(suffix)
}

get_suffix(mem) = suffix {
	is_string(mem)
	count(mem) > 1
	suffix := substring(mem, count(mem) - 2, -1)
	mem_multiple(suffix)
}

get_suffix(mem) = suffix {
	is_string(mem)
	count(mem) > 1
	not mem_multiple(substring(mem, count(mem) - 1, -1))
	not mem_multiple(substring(mem, count(mem) - 2, -1))
	suffix := ""
}

get_suffix(mem) = suffix {
	is_string(mem)
	count(mem) == 1
	not mem_multiple(substring(mem, count(mem) - 1, -1))
	suffix := ""
}

get_suffix(mem) = suffix {
	is_string(mem)
	count(mem) == 0
	suffix := ""
}

canonify_mem(orig) = new {
	is_number(orig)
	new := orig * 1000
}

canonify_mem(orig) = new {
	not is_number(orig)
	suffix := get_suffix(orig)
	raw := replace(orig, suffix, "")
	re_match("^[0-9]+$", raw)
	new := to_number(raw) * mem_multiple(suffix)
}

violation[{"msg": msg}] {
	general_violation[{"msg": msg, "field": "containers"}]
}

violation[{"msg": msg}] {
	general_violation[{"msg": msg, "field": "initContainers"}]
}

general_violation[{"msg": msg, "field": field}] {
	container := input.review.object.spec[field][_]
	cpu_orig := container.resources.limits.cpu
	not canonify_cpu(cpu_orig)
	msg := sprintf("container <%v> cpu limit <%v> could not be parsed", [container.name, cpu_orig])
}

general_violation[{"msg": msg, "field": field}] {
	container := input.review.object.spec[field][_]
	mem_orig := container.resources.limits.memory
	not canonify_mem(mem_orig)
	msg := sprintf("container <%v> memory limit <%v> could not be parsed", [container.name, mem_orig])
}

general_violation[{"msg": msg, "field": field}] {
	container := input.review.object.spec[field][_]
	not container.resources
	msg := sprintf("container <%v> has no resource limits", [container.name])
}

general_violation[{"msg": msg, "field": field}] {
	container := input.review.object.spec[field][_]
	not container.resources.limits
	msg := sprintf("container <%v> has no resource limits", [container.name])
}

general_violation[{"msg": msg, "field": field}] {
	container := input.review.object.spec[field][_]
	missing(container.resources.limits, "cpu")
	msg := sprintf("container <%v> has no cpu limit", [container.name])
}

general_violation[{"msg": msg, "field": field}] {
	container := input.review.object.spec[field][_]
	missing(container.resources.limits, "memory")
	msg := sprintf("container <%v> has no memory limit", [container.name])
}

general_violation[{"msg": msg, "field": field}] {
	container := input.review.object.spec[field][_]
	cpu_orig := container.resources.limits.cpu
	cpu := canonify_cpu(cpu_orig)
	max_cpu_orig := input.parameters.cpu
	max_cpu := canonify_cpu(max_cpu_orig)
	cpu > max_cpu
	msg := sprintf("container <%v> cpu limit <%v> is higher than the maximum allowed of <%v>", [container.name, cpu_orig, max_cpu_orig])
}

general_violation[{"msg": msg, "field": field}] {
	container := input.review.object.spec[field][_]
	mem_orig := container.resources.limits.memory
	mem := canonify_mem(mem_orig)
	max_mem_orig := input.parameters.memory
	max_mem := canonify_mem(max_mem_orig)
	mem > max_mem
	msg := sprintf("container <%v> memory limit <%v> is higher than the maximum allowed of <%v>", [container.name, mem_orig, max_mem_orig])
}
""")

REQUIRED_PROBES = _tmpl("K8sRequiredProbes", """package k8srequiredprobes

probe_type_set = probe_types {
	probe_types := {type | type := input.parameters.probeTypes[_]}
}

violation[{"msg": msg}] {
	container := input.review.object.spec.containers[_]
	probe := input.parameters.probes[_]
	probe_is_missing(container, probe)
	msg := get_violation_message(container, input.review, probe)
}

probe_is_missing(ctr, probe) = true {
	not ctr[probe]
}

probe_is_missing(ctr, probe) = true {
	probe_field_empty(ctr, probe)
}

probe_field_empty(ctr, probe) = true {
	probe_fields := {field | ctr[probe][field]}
	diff_fields := probe_type_set - probe_fields
	count(diff_fields) == count(probe_type_set)
}

get_violation_message(container, review, probe) = msg {
	msg := sprintf("Container <%v> in your <%v> <%v> has no <%v>", [container.name, review.kind.kind, review.object.metadata.name, probe])
}
""")

# demo/agilebank/templates/k8suniqueserviceselector_template.yaml: a
# data.inventory join (outside the GPU subset).  The engine compiles it as a
# guard program: the three `input.review.kind` tests run on the device, so only
# v1 Services reach the inventory join and go to the CPU.
UNIQUE_SERVICE_SELECTOR = _tmpl("K8sUniqueServiceSelector", """package k8suniqueserviceselector

make_apiversion(kind) = apiVersion {
	g := kind.group
	v := kind.version
	g != ""
	apiVersion = sprintf("%v/%v", [g, v])
}

make_apiversion(kind) = apiVersion {
	kind.group == ""
	apiVersion = kind.version
}

identical(obj, review) {
	obj.metadata.namespace == review.namespace
	obj.metadata.name == review.name
	obj.kind == review.kind.kind
	obj.apiVersion == make_apiversion(review.kind)
}

flatten_selector(obj) = flattened {
	selectors := [s | s = concat(":", [key, val]); val = obj.spec.selector[key]]
	flattened := concat(",", sort(selectors))
}

violation[{"msg": msg}] {
	input.review.kind.kind == "Service"
	input.review.kind.version == "v1"
	input.review.kind.group == ""
	input_selector := flatten_selector(input.review.object)
	other := data.inventory.namespace[namespace][_][_][name]
	not identical(other, input.review)
	other_selector := flatten_selector(other)
	input_selector == other_selector
	msg := sprintf("same selector as service <%v> in namespace <%v>", [name, namespace])
}
""")

# demo/agilebank/dryrun/k8suniqueingresshost_template.yaml: the third
# data.inventory join of the reference (a multi-valued key: every rule host)
UNIQUE_INGRESS_HOST = _tmpl("K8sUniqueIngressHost", """package k8suniqueingresshost

identical(obj, review) {
	obj.metadata.namespace == review.object.metadata.namespace
	obj.metadata.name == review.object.metadata.name
}

violation[{"msg": msg}] {
	input.review.kind.kind == "Ingress"
	re_match("^(extensions|networking.k8s.io)$", input.review.kind.group)
	host := input.review.object.spec.rules[_].host
	other := data.inventory.namespace[ns][otherapiversion]["Ingress"][name]
	re_match("^(extensions|networking.k8s.io)/.+$", otherapiversion)
	other.spec.rules[_].host == host
	not identical(other, input.review)
	msg := sprintf("ingress host conflicts with an existing ingress <%v>", [host])
}
""")


def gen_ingresses(n, seed=5, n_namespaces=20, n_hosts=None):
    """n Ingresses (extensions/v1beta1 and networking.k8s.io/v1beta1, one in
    eight under another group) with 1-3 rule hosts each drawn from n_hosts
    names (default n // 2, so hosts collide), over n_namespaces namespaces.
    (objects, their Namespaces)"""
    k = n_hosts or max(1, n // 2)
    r = random.Random(seed)
    names = ["ing-ns-%02d" % i for i in range(n_namespaces)]
    objs, nss = [], []
    for i in range(n):
        ns = names[r.randrange(n_namespaces)]
        av = ("extensions/v1beta1", "networking.k8s.io/v1beta1", "example.com/v1")[2 if i % 8 == 7 else i % 2]
        rules = [{"host": "h%d.example.com" % r.randrange(k)} for _ in range(1 + r.randrange(3))]
        if i % 11 == 0:
            rules.append({"http": {"paths": []}})  # a rule without a host
        objs.append({"apiVersion": av, "kind": "Ingress", "metadata": {"name": "ing-%05d" % i, "namespace": ns},
                     "spec": {"rules": rules}})
        nss.append(namespace_obj(ns))
    return objs, nss


ALLOWED_LABEL_REGEX = _tmpl("K8sAllowedLabelRegex", """package k8sallowedlabelregex

violation[{"msg": msg, "details": {"label": key}}] {
	value := input.review.object.metadata.labels[key]
	rule := input.parameters.rules[_]
	rule.key == key
	not re_match(rule.allowedRegex, value)
	msg := sprintf("label <%v: %v> does not match allowed regex %v", [key, value, rule.allowedRegex])
}
""")

ALLOWED_ANNOTATION_REGEX = _tmpl("K8sAllowedAnnotationRegex", """package k8sallowedannotationregex

violation[{"msg": msg, "details": {"annotation": key}}] {
	value := input.review.object.metadata.annotations[key]
	rule := input.parameters.rules[_]
	rule.key == key
	not re_match(rule.allowedRegex, value)
	msg := sprintf("annotation <%v: %v> does not match allowed regex %v", [key, value, rule.allowedRegex])
}
""")


# demo/basic/templates/k8suniquelabel_template.yaml: a label value must be
# unique across the synced inventory (data.inventory join + array.concat)
UNIQUE_LABEL = _tmpl("K8sUniqueLabel", """package k8suniquelabel

make_apiversion(kind) = apiVersion {
	g := kind.group
	v := kind.version
	g != ""
	apiVersion = sprintf("%v/%v", [g, v])
}

make_apiversion(kind) = apiVersion {
	kind.group == ""
	apiVersion = kind.version
}

identical_namespace(obj, review) {
	obj.metadata.namespace == review.namespace
	obj.metadata.name == review.name
	obj.kind == review.kind.kind
	obj.apiVersion == make_apiversion(review.kind)
}

identical_cluster(obj, review) {
	obj.metadata.name == review.name
	obj.kind == review.kind.kind
	obj.apiVersion == make_apiversion(review.kind)
}

violation[{"msg": msg, "details": {"value": val, "label": label}}] {
	label := input.parameters.label
	val := input.review.object.metadata.labels[label]
	cluster_objs := [o | o = data.inventory.cluster[_][_][_]; not identical_cluster(o, input.review)]
	ns_objs := [o | o = data.inventory.namespace[_][_][_][_]; not identical_namespace(o, input.review)]
	all_objs := array.concat(cluster_objs, ns_objs)
	all_values := {val | obj = all_objs[_]; val = obj.metadata.labels[label]}
	count({val} - all_values) == 0
	msg := sprintf("label %v has duplicate value %v", [label, val])
}
""", {"properties": {"label": {"type": "string"}}})


def constraint(kind, name, match=None, parameters=None, enforcement_action=None):
    spec = {}
    if match is not None:
        spec["match"] = match
    if parameters is not None:
        spec["parameters"] = parameters
    if enforcement_action is not None:
        spec["enforcementAction"] = enforcement_action
    c = {"apiVersion": "constraints.gatekeeper.sh/v1beta1", "kind": kind, "metadata": {"name": name}}
    if spec:
        c["spec"] = spec
    return c


# -- config 1: demo/basic all_ns_must_have_gatekeeper.yaml over namespaces
def config1():
    templates = [REQUIRED_LABELS_BASIC]
    constraints = [constraint("K8sRequiredLabels", "ns-must-have-gk",
                              match={"kinds": [{"apiGroups": [""], "kinds": ["Namespace"]}]},
                              parameters={"labels": ["gatekeeper"]})]
    return templates, constraints


# -- config 2: demo/agilebank constraints (demo/agilebank/constraints/*.yaml) over Pods
def config2():
    """The five demo/agilebank constraints.  unique-service-selector has no
    match block (demo/agilebank/constraints/unique_service_selector.yaml), so it
    matches every review; its template is served by a guard program (see
    UNIQUE_SERVICE_SELECTOR) and no Pod falls back."""
    templates, constraints = config2_gpu_subset()
    templates.append(UNIQUE_SERVICE_SELECTOR)
    constraints.append({"apiVersion": "constraints.gatekeeper.sh/v1beta1", "kind": "K8sUniqueServiceSelector",
                        "metadata": {"name": "unique-service-selector", "labels": {"owner": "admin.agilebank.demo"}}})
    return templates, constraints


def config2_gpu_subset():
    """config 2 without unique-service-selector: the four templates inside the GPU subset."""
    templates = [REQUIRED_LABELS, ALLOWED_REPOS, CONTAINER_LIMITS, REQUIRED_PROBES]
    constraints = [
        constraint("K8sRequiredLabels", "all-must-have-owner",
                   match={"kinds": [{"apiGroups": [""], "kinds": ["Namespace"]}]},
                   parameters={"message": "All namespaces must have an `owner` label that points to your company username",
                               "labels": [{"key": "owner", "allowedRegex": "^[a-zA-Z]+.agilebank.demo$"}]}),
        constraint("K8sAllowedRepos", "prod-repo-is-openpolicyagent",
                   match={"kinds": [{"apiGroups": [""], "kinds": ["Pod"]}], "namespaces": ["production"]},
                   parameters={"repos": ["openpolicyagent"]}),
        constraint("K8sContainerLimits", "container-must-have-limits",
                   match={"kinds": [{"apiGroups": [""], "kinds": ["Pod"]}]},
                   parameters={"cpu": "200m", "memory": "1Gi"}),
        constraint("K8sRequiredProbes", "must-have-probes",
                   match={"kinds": [{"apiGroups": [""], "kinds": ["Pod"]}]},
                   parameters={"probes": ["readinessProbe", "livenessProbe"], "probeTypes": ["tcpSocket", "httpGet", "exec"]}),
    ]
    return templates, constraints


_ALNUM = "abcdefghijklmnopqrstuvwxyz0123456789"


def _word(rng, lo=1, hi=16, alphabet=_ALNUM + "-"):
    n = rng.randint(lo, hi)
    s = "".join(rng.choice(alphabet) for _ in range(n))
    return s


def namespace_obj(name, labels=None):
    md = {"name": name, "creationTimestamp": None}
    if labels:
        md["labels"] = labels
    return {"apiVersion": "v1", "kind": "Namespace", "metadata": md, "spec": {"finalizers": ["kubernetes"]},
            "status": {"phase": "Active"}}


def gen_namespaces(n, seed=1):
    """Config 1: `ns-%05d`, P(gatekeeper label)=0.5, plus 0-3 labels from a 64-key vocabulary."""
    rng = random.Random(seed)
    vocab = ["k%02d-%s" % (i, _word(rng, 3, 8, _ALNUM)) for i in range(64)]
    out = []
    for i in range(n):
        labels = {}
        if rng.random() < 0.5:
            labels["gatekeeper"] = _word(rng, 1, 16)
        for _ in range(rng.randint(0, 3)):
            labels[rng.choice(vocab)] = _word(rng, 1, 16)
        if rng.random() < 0.3:
            labels["owner"] = rng.choice(["alice.agilebank.demo", "bob", "x.agilebank.demo", "Carol1.agilebank.demo"])
        out.append(namespace_obj("ns-%05d" % i, labels or None))
    return out


_CPU = ["100m", "200m", "300m", "1", "0.5", "2000m", None]
_MEMV = ["30Mi", "1Gi", "4000Mi", "2G", "512Ki", None]


def gen_pods(n, seed=42, n_namespaces=1000):
    """Config 2: Pods over 1,000 namespaces (10% named `production`), 1-4 containers +
    0-1 initContainers, images from {openpolicyagent/opa 60%, gcr.io/x/opa 20%, nginx 20%},
    cpu/memory limits from SURVEY 8(d)'s value sets, probes P=0.5, `owner` label P=0.7."""
    rng = random.Random(seed)
    nss = []
    for i in range(n_namespaces):
        name = "production" if i < n_namespaces // 10 else "team-%04d" % i
        if name == "production" and i > 0:
            name = "production-%03d" % i
        nss.append(name)
    # 10% of namespaces are "production": only one literal name can equal it, so
    # route 10% of pods there explicitly
    objs, ns_of = [], []
    ns_objs = {}
    for i in range(n):
        ns = "production" if rng.random() < 0.10 else rng.choice(nss[n_namespaces // 10:] or ["default"])
        conts = []
        for c in range(rng.randint(1, 4)):
            conts.append(_container(rng, "c%d" % c))
        pod_spec = {"containers": conts}
        if rng.random() < 0.5:
            pod_spec["initContainers"] = [_container(rng, "init")]
        labels = {"app": "app-%d" % rng.randint(0, 99)}
        if rng.random() < 0.7:
            labels["owner"] = rng.choice(["alice", "bob.agilebank.demo"])
        obj = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": "pod-%07d" % i, "namespace": ns, "labels": labels}, "spec": pod_spec}
        objs.append(obj)
        if ns not in ns_objs:
            ns_objs[ns] = namespace_obj(ns, {"env": "prod" if ns == "production" else "dev"})
        ns_of.append(ns)
    return objs, ns_of, ns_objs


def _container(rng, name):
    r = rng.random()
    tag = "0.%d.%d" % (rng.randint(1, 30), rng.randint(0, 9))
    if r < 0.6:
        image = "openpolicyagent/opa:" + tag
    elif r < 0.8:
        image = "gcr.io/x/opa:" + tag
    else:
        image = "nginx"
    c = {"name": name, "image": image}
    cpu = rng.choice(_CPU)
    mem = rng.choice(_MEMV)
    if cpu is not None or mem is not None or rng.random() < 0.5:
        lim = {}
        if cpu is not None:
            lim["cpu"] = cpu
        if mem is not None:
            lim["memory"] = mem
        c["resources"] = {"limits": lim}
    for probe in ("readinessProbe", "livenessProbe"):
        if rng.random() < 0.5:
            kind = rng.choice(["tcpSocket", "httpGet", "exec", "other"])
            c[probe] = {kind: {"port": 8080}} if kind != "other" else {"initialDelaySeconds": 3}
    return c


def dumps(x) -> str:
    return json.dumps(x, separators=(",", ":"))


def gen_pods_json(n, seed=42, n_namespaces=1000, start=0):
    """Fast JSON-text generator with gen_pods' distribution (config 2 at scale).

    Returns (object JSON strings, namespace JSON strings aligned with objects);
    namespace strings are shared objects per namespace.  Containers are drawn
    from seeded pools of pre-serialized variants (2,048 per slot)."""
    rng = random.Random(seed)
    pools = [[json.dumps(_container(rng, "c%d" % slot), separators=(",", ":")) for _ in range(2048)] for slot in range(4)]
    init_pool = [json.dumps(_container(rng, "init"), separators=(",", ":")) for _ in range(2048)]
    names = ["team-%04d" % i for i in range(n_namespaces - 1)]
    ns_json = {nm: dumps(namespace_obj(nm, {"env": "dev"})) for nm in names}
    ns_json["production"] = dumps(namespace_obj("production", {"env": "prod"}))
    objs, nss = [], []
    r = random.Random(seed * 7919 + start)
    rand = r.random
    rbits = r.getrandbits
    for i in range(start, start + n):
        ns = "production" if rand() < 0.10 else names[rbits(16) % len(names)]
        k = 1 + (rbits(2))
        conts = ",".join(pools[s][rbits(11)] for s in range(k))
        init = (',"initContainers":[' + init_pool[rbits(11)] + "]") if rand() < 0.5 else ""
        owner = (',"owner":"alice"' if rand() < 0.5 else ',"owner":"bob.agilebank.demo"') if rand() < 0.7 else ""
        objs.append('{"apiVersion":"v1","kind":"Pod","metadata":{"name":"pod-%08d","namespace":"%s","labels":{"app":"app-%d"%s}},'
                    '"spec":{"containers":[%s]%s}}' % (i, ns, rbits(7), owner, conts, init))
        nss.append(ns_json[ns])
    return objs, nss


# -- config 3: allowedRegex label / annotation templates over Deployments + Services
_C3_RULES = {
    "env": "^(dev|stage|prod)-[0-9]{1,4}$",
    "owner": "^[a-zA-Z]+.agilebank.demo$",
    "app": "^[a-z0-9]([-a-z0-9]*[a-z0-9])?$",
    "tier": "^(frontend|backend|cache|db)$",
    "team": "^team-[a-z]{2,8}$",
    "version": "^v[0-9]+\\.[0-9]+\\.[0-9]+$",
    "region": "^[a-z]{2}-[a-z]+-[0-9]$",
    "component": "^[a-z]+(-[a-z]+)*$",
    # Go RE2 specifics (round 6): `\s` is [\t\n\f\r ] (no \v), and (?i) folds
    # k with U+212A (KELVIN SIGN) and s with U+017F (LONG S); neither pattern is
    # utf8-sensitive (no `.`, no negated class), so the device decides every
    # value, non-ASCII ones included
    "note": "^[a-z]+(\\s[a-z0-9]+)*$",
    "kube": "(?i)^(kube|sys)-[a-z]+$",
}
# config 4 keeps the first eight (its workload is unchanged since round 4)
_C3_BASE_KEYS = ("env", "owner", "app", "tier", "team", "version", "region", "component")
# values near each pattern's boundaries (~half match); no value needs the
# UTF-8 fallback: the non-ASCII ones are only checked by non-sensitive patterns
_C3_VALUES = {
    "env": ["dev-1", "prod-9999", "stage-42", "prod-10000", "stage-", "dev-12\n", "qa-1", "", "DEV-1", "prod-0001"],
    "owner": ["alice.agilebank.demo", "Bob.agilebank.demo", "bob_agilebank.demo", "x.agilebank.demo\n",
              "9.agilebank.demo", "carol-agilebank-demo", "dave.agilebank.demo.", "e.agilebankXdemo"],
    "app": ["web", "-web", "web-", "a", "Web", "a-b-c", "", "api-7", "x" * 40, "db_1"],
    "tier": ["frontend", "backend", "cache", "db", "Frontend", "frontend ", "web", ""],
    "team": ["team-ab", "team-payments", "team-a", "team-abcdefghi", "Team-ab", "team-12", "team-ops"],
    "version": ["v1.2.3", "v10.0.1", "1.2.3", "v1.2", "v1.2.3-rc1", "v01.2.3", "v1..3"],
    "region": ["us-east-1", "eu-west-2", "us-east-12", "US-east-1", "ap-south", "eu-central-3"],
    "component": ["api", "api-server", "-api", "api-", "API", "a-b-c-d", "api--server"],
    "note": ["ok go", "ok\tgo", "ok\vgo", "ok\ngo", "ok  go", "ok go\v", "ok", "ok\r\n1", "x\x0cy", "ok\u00a0go"],
    "kube": ["kube-ops", "KUBE-ops", "\u212aube-ops", "\u017fys-x", "kube-\u212a\u017f", "kube-", "ube-x",
             "\u0130kube-x", "sys-\u00e9", "SYS-OK"],
}


def config3():
    """10 allowedRegex constraints: 5 over labels, 5 over annotations, each a
    different pair of key rules, all matching Deployments and Services."""
    keys = list(_C3_RULES)
    cs = []
    for i in range(5):
        sel = [keys[(2 * i + j) % len(keys)] for j in range(3)]
        rules = [{"key": k, "allowedRegex": _C3_RULES[k]} for k in sel]
        match = {"kinds": [{"apiGroups": ["apps", ""], "kinds": ["Deployment", "Service"]}]}
        cs.append(constraint("K8sAllowedLabelRegex", "label-rules-%d" % i, match=match, parameters={"rules": rules}))
        cs.append(constraint("K8sAllowedAnnotationRegex", "annotation-rules-%d" % i, match=match,
                             parameters={"rules": rules}))
    return [ALLOWED_LABEL_REGEX, ALLOWED_ANNOTATION_REGEX], cs


def gen_config3_json(n, seed=7, start=0, n_namespaces=200):
    """Config 3 at scale: 50% Deployments / 50% Services, 2-8 labels and 0-4
    annotations drawn from _C3_VALUES (JSON text; pools of pre-serialized maps)."""
    rng = random.Random(seed)
    keys = list(_C3_VALUES)

    def amap(lo, hi):
        ks = rng.sample(keys, rng.randint(lo, hi))
        return {k: rng.choice(_C3_VALUES[k]) for k in ks}

    lab_pool = [dumps(amap(2, 8)) for _ in range(4096)]
    ann_pool = [dumps(amap(0, 4)) for _ in range(4096)]
    names = ["c3-ns-%03d" % i for i in range(n_namespaces)]
    ns_json = {nm: dumps(namespace_obj(nm, {"env": "dev"})) for nm in names}
    r = random.Random(seed * 7919 + start)
    rb = r.getrandbits
    objs, nss = [], []
    for i in range(start, start + n):
        ns = names[rb(16) % len(names)]
        lab, ann = lab_pool[rb(12)], ann_pool[rb(12)]
        if rb(1):
            objs.append('{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"dep-%08d","namespace":"%s",'
                        '"labels":%s,"annotations":%s},"spec":{"replicas":%d}}' % (i, ns, lab, ann, 1 + rb(3)))
        else:
            objs.append('{"apiVersion":"v1","kind":"Service","metadata":{"name":"svc-%08d","namespace":"%s",'
                        '"labels":%s,"annotations":%s},"spec":{"ports":[{"port":%d}]}}' % (i, ns, lab, ann, 80 + rb(10)))
        nss.append(ns_json[ns])
    return objs, nss


# -- config 6 (VERDICT r02 "next" #6): config 2 with its data.inventory joins
# exercised -- Services and labelled Deployments synced into the inventory and
# reviewed by the audit, unique-service-selector (agilebank) and a
# unique-label constraint (demo/basic) over them
def config6():
    templates, constraints = config2()
    templates = templates + [UNIQUE_LABEL]
    constraints = constraints + [constraint(
        "K8sUniqueLabel", "deployment-app-label-unique",
        match={"kinds": [{"apiGroups": ["apps"], "kinds": ["Deployment"]}]}, parameters={"label": "app"})]
    return templates, constraints


def gen_config6_json(n, seed=11, start=0, n_namespaces=100, n_selectors=None):
    """n objects, half Services (spec.selector {app, tier?}) and half
    Deployments (metadata.labels.app), over n_namespaces namespaces; selector
    and label values repeat (n_selectors distinct, default n // 4), so the
    joins find duplicates.  JSON text, with each object's Namespace."""
    k = n_selectors or max(1, n // 4)
    names = ["j-ns-%03d" % i for i in range(n_namespaces)]
    ns_json = {nm: dumps(namespace_obj(nm)) for nm in names}
    r = random.Random(seed * 7919 + start)
    rb = r.getrandbits
    objs, nss = [], []
    for i in range(start, start + n):
        ns = names[rb(16) % len(names)]
        app = "app-%d" % (rb(30) % k)
        if i % 2 == 0:
            sel = '{"app":"%s"}' % app if rb(2) else '{"app":"%s","tier":"%s"}' % (app, ("web", "db")[rb(1)])
            objs.append('{"apiVersion":"v1","kind":"Service","metadata":{"name":"svc-%08d","namespace":"%s"},'
                        '"spec":{"selector":%s,"ports":[{"port":80}]}}' % (i, ns, sel))
        else:
            objs.append('{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"dep-%08d","namespace":"%s",'
                        '"labels":{"app":"%s"}},"spec":{"replicas":1}}' % (i, ns, app))
        nss.append(ns_json[ns])
    return objs, nss


def inventory_paths(objs_json):
    """(data path, object JSON) of synced objects (client.data_path:
    K8sValidationTarget.ProcessData, pkg/target/target.go:62-76)"""
    from .client import data_path
    return [(data_path(json.loads(js)), js) for js in objs_json]


# -- config 4: 50 constraints cloned from the subset templates, randomized match
_C4_KINDS = [("", "Pod"), ("apps", "Deployment"), ("", "Service"), ("", "ConfigMap"), ("", "Namespace")]


def config4(seed=1234, n_namespaces=1000):
    """50 constraints over the subset templates with randomized match (kinds,
    namespaces, excludedNamespaces, labelSelector In/NotIn/Exists/DoesNotExist,
    namespaceSelector, scope) and parameters."""
    rng = random.Random(seed)
    ns_names = ["team-%04d" % i for i in range(n_namespaces - 1)] + ["production"]
    templates = [REQUIRED_LABELS, ALLOWED_REPOS, CONTAINER_LIMITS, REQUIRED_PROBES, ALLOWED_LABEL_REGEX,
                 ALLOWED_ANNOTATION_REGEX]
    cs = []
    for i in range(50):
        kind = ["K8sRequiredLabels", "K8sAllowedRepos", "K8sContainerLimits", "K8sRequiredProbes",
                "K8sAllowedLabelRegex", "K8sAllowedAnnotationRegex"][i % 6]
        match = {}
        r = rng.random()
        if r < 0.15:
            pass  # default kinds: everything
        else:
            ks = rng.sample(_C4_KINDS, rng.randint(1, 3))
            groups = sorted({g for g, _ in ks})
            match["kinds"] = [{"apiGroups": groups if rng.random() < 0.7 else ["*"], "kinds": [k for _, k in ks]}]
        if rng.random() < 0.2:
            match["namespaces"] = rng.sample(ns_names, 3) + ["production"]
        if rng.random() < 0.2:
            match["excludedNamespaces"] = rng.sample(ns_names, 5)
        if rng.random() < 0.3:
            op = rng.choice(["In", "NotIn", "Exists", "DoesNotExist"])
            e = {"key": rng.choice(["app", "owner", "tier"]), "operator": op}
            if op in ("In", "NotIn"):
                e["values"] = ["app-%d" % rng.randint(0, 99) for _ in range(3)] + ["alice", "frontend"]
            sel = {"matchExpressions": [e]}
            if rng.random() < 0.3:
                sel["matchLabels"] = {"app": "app-%d" % rng.randint(0, 9)}
            match["labelSelector"] = sel
        if rng.random() < 0.25:
            match["namespaceSelector"] = {"matchExpressions": [
                {"key": "env", "operator": rng.choice(["In", "NotIn"]), "values": [rng.choice(["dev", "prod", "stage"])]}]}
        if rng.random() < 0.15:
            match["scope"] = rng.choice(["Namespaced", "Cluster", "*"])
        if kind == "K8sRequiredLabels":
            params = {"labels": [{"key": rng.choice(["owner", "app", "tier"]),
                                  "allowedRegex": rng.choice(["^[a-zA-Z]+.agilebank.demo$", "^app-[0-9]+$", ""])}]}
            if rng.random() < 0.5:
                params["message"] = "constraint %d: required label missing" % i
        elif kind == "K8sAllowedRepos":
            params = {"repos": rng.sample(["openpolicyagent", "gcr.io/x", "nginx", "docker.io/library"], 2)}
        elif kind == "K8sContainerLimits":
            params = {"cpu": rng.choice(["100m", "200m", "1", "2"]), "memory": rng.choice(["512Mi", "1Gi", "2Gi", "1G"])}
        elif kind == "K8sRequiredProbes":
            params = {"probes": rng.sample(["readinessProbe", "livenessProbe"], rng.randint(1, 2)),
                      "probeTypes": ["tcpSocket", "httpGet", "exec"]}
        else:
            keys = rng.sample(list(_C3_BASE_KEYS), 2)
            params = {"rules": [{"key": k, "allowedRegex": _C3_RULES[k]} for k in keys]}
        ea = "dryrun" if rng.random() < 0.2 else None
        cs.append(constraint(kind, "c4-%02d-%s" % (i, kind.lower()), match=match or None, parameters=params,
                             enforcement_action=ea))
    return templates, cs


def gen_config4_json(n, seed=1234, start=0, n_namespaces=1000):
    """Config 4 mix: Pods 60%, Deployments 15%, Services 10%, ConfigMaps 14%,
    Namespaces 1% (cluster-scoped: no namespace object)."""
    rng = random.Random(seed)
    pools = [[dumps(_container(rng, "c%d" % slot)) for _ in range(1024)] for slot in range(4)]
    init_pool = [dumps(_container(rng, "init")) for _ in range(1024)]
    keys = list(_C3_BASE_KEYS)

    def labels():
        d = {"app": "app-%d" % rng.randint(0, 99)}
        if rng.random() < 0.6:
            d["owner"] = rng.choice(["alice", "bob.agilebank.demo", "Carol.agilebank.demo"])
        if rng.random() < 0.5:
            d["tier"] = rng.choice(_C3_VALUES["tier"])
        for k in rng.sample(keys, rng.randint(0, 2)):
            d[k] = rng.choice(_C3_VALUES[k])
        return dumps(d)

    lab_pool = [labels() for _ in range(4096)]
    ann_pool = [dumps({k: rng.choice(_C3_VALUES[k]) for k in rng.sample(keys, rng.randint(0, 3))}) for _ in range(1024)]
    names = ["team-%04d" % i for i in range(n_namespaces - 1)] + ["production"]
    envs = ["dev", "prod", "stage"]
    ns_json = {nm: dumps(namespace_obj(nm, {"env": "prod" if nm == "production" else envs[sum(map(ord, nm)) % 3]}))
               for nm in names}
    r = random.Random(seed * 7919 + start)
    rand, rb = r.random, r.getrandbits
    objs, nss = [], []
    for i in range(start, start + n):
        ns = names[rb(16) % len(names)]
        lab, ann = lab_pool[rb(12)], ann_pool[rb(10)]
        x = rand()
        k = 1 + rb(2)
        conts = ",".join(pools[s][rb(10)] for s in range(k))
        if x < 0.60:
            init = (',"initContainers":[' + init_pool[rb(10)] + "]") if rand() < 0.3 else ""
            objs.append('{"apiVersion":"v1","kind":"Pod","metadata":{"name":"pod-%08d","namespace":"%s","labels":%s,'
                        '"annotations":%s},"spec":{"containers":[%s]%s}}' % (i, ns, lab, ann, conts, init))
        elif x < 0.75:
            objs.append('{"apiVersion":"apps/v1","kind":"Deployment","metadata":{"name":"dep-%08d","namespace":"%s",'
                        '"labels":%s,"annotations":%s},"spec":{"replicas":%d,"template":{"metadata":{"labels":%s},'
                        '"spec":{"containers":[%s]}}}}' % (i, ns, lab, ann, 1 + rb(3), lab, conts))
        elif x < 0.85:
            objs.append('{"apiVersion":"v1","kind":"Service","metadata":{"name":"svc-%08d","namespace":"%s","labels":%s,'
                        '"annotations":%s},"spec":{"selector":%s,"ports":[{"port":%d}]}}' % (i, ns, lab, ann, lab, 80 + rb(8)))
        elif x < 0.99:
            objs.append('{"apiVersion":"v1","kind":"ConfigMap","metadata":{"name":"cm-%08d","namespace":"%s","labels":%s},'
                        '"data":{"k":"v%d"}}' % (i, ns, lab, rb(10)))
        else:
            objs.append('{"apiVersion":"v1","kind":"Namespace","metadata":{"name":"nsobj-%08d","labels":%s},'
                        '"spec":{"finalizers":["kubernetes"]},"status":{"phase":"Active"}}' % (i, lab))
            nss.append(None)
            continue
        nss.append(ns_json[ns])
    return objs, nss


# -- config 5: admission-webhook micro-batch over the PSP policies of
# BenchmarkValidationHandler (pkg/webhook/policy_benchmark_test.go:233-329;
# templates/constraints/pods from pkg/webhook/testdata/psp-all-violations/)
PSP_HOST_FILESYSTEM = _tmpl("K8sPSPHostFilesystem", """package k8spsphostfilesystem

violation[{"msg": msg, "details": {}}] {
	volume := input_hostpath_volumes[_]
	not input_hostpath_allowed(volume)
	msg := sprintf("HostPath volume %v is not allowed, pod: %v. Allowed path: %v", [volume, input.review.object.metadata.name, input.parameters.allowedHostPaths])
}

input_hostpath_allowed(volume) {
	input.parameters.allowedHostPaths == []
}

input_hostpath_allowed(volume) {
	allowedHostPath := input.parameters.allowedHostPaths[_]
	path_matches(allowedHostPath.pathPrefix, volume.hostPath.path)
	not allowedHostPath.readOnly == true
}

input_hostpath_allowed(volume) {
	allowedHostPath := input.parameters.allowedHostPaths[_]
	path_matches(allowedHostPath.pathPrefix, volume.hostPath.path)
	allowedHostPath.readOnly
	not writeable_input_volume_mounts(volume.name)
}

writeable_input_volume_mounts(volume_name) {
	container := input_containers[_]
	mount := container.volumeMounts[_]
	mount.name == volume_name
	not mount.readOnly
}

path_matches(prefix, path) {
	a := split(trim(prefix, "/"), "/")
	b := split(trim(path, "/"), "/")
	prefix_matches(a, b)
}

prefix_matches(a, b) {
	count(a) <= count(b)
	not any_not_equal_upto(a, b, count(a))
}

any_not_equal_upto(a, b, n) {
	a[i] != b[i]
	i < n
}

input_hostpath_volumes[v] {
	v := input.review.object.spec.volumes[_]
	has_field(v, "hostPath")
}

has_field(object, field) = true {
	object[field]
}

input_containers[c] {
	c := input.review.object.spec.containers[_]
}

input_containers[c] {
	c := input.review.object.spec.initContainers[_]
}
""")

PSP_HOST_NAMESPACE = _tmpl("K8sPSPHostNamespace", """package k8spsphostnamespace

violation[{"msg": msg, "details": {}}] {
	input_share_hostnamespace(input.review.object)
	msg := sprintf("Sharing the host namespace is not allowed: %v", [input.review.object.metadata.name])
}

input_share_hostnamespace(o) {
	o.spec.hostPID
}

input_share_hostnamespace(o) {
	o.spec.hostIPC
}
""")

PSP_HOST_NETWORK_PORTS = _tmpl("K8sPSPHostNetworkingPorts", """package k8spsphostnetworkingports

violation[{"msg": msg, "details": {}}] {
	input_share_hostnetwork(input.review.object)
	msg := sprintf("The specified hostNetwork and hostPort are not allowed, pod: %v. Allowed values: %v", [input.review.object.metadata.name, input.parameters])
}

input_share_hostnetwork(o) {
	not input.parameters.hostNetwork
	o.spec.hostNetwork
}

input_share_hostnetwork(o) {
	hostPort := input_containers[_].ports[_].hostPort
	hostPort < input.parameters.min
}

input_share_hostnetwork(o) {
	hostPort := input_containers[_].ports[_].hostPort
	hostPort > input.parameters.max
}

input_containers[c] {
	c := input.review.object.spec.containers[_]
}

input_containers[c] {
	c := input.review.object.spec.initContainers[_]
}
""")

PSP_PRIVILEGED = _tmpl("K8sPSPPrivilegedContainer", """package k8spspprivileged

violation[{"msg": msg, "details": {}}] {
	c := input_containers[_]
	c.securityContext.privileged
	msg := sprintf("Privileged container is not allowed: %v, securityContext: %v", [c.name, c.securityContext])
}

input_containers[c] {
	c := input.review.object.spec.containers[_]
}

input_containers[c] {
	c := input.review.object.spec.initContainers[_]
}
""")

PSP_VOLUME_TYPES = _tmpl("K8sPSPVolumeTypes", """package k8spspvolumetypes

violation[{"msg": msg, "details": {}}] {
	volume_fields := {x | input.review.object.spec.volumes[_][x]; x != "name"}
	not input_volume_type_allowed(volume_fields)
	msg := sprintf("One of the volume types %v is not allowed, pod: %v. Allowed volume types: %v", [volume_fields, input.review.object.metadata.name, input.parameters.volumes])
}

input_volume_type_allowed(volume_fields) {
	input.parameters.volumes[_] == "*"
}

input_volume_type_allowed(volume_fields) {
	allowed_set := {x | x = input.parameters.volumes[_]}
	test := volume_fields - allowed_set
	count(test) == 0
}
""")

PSP_TEMPLATES = [PSP_HOST_FILESYSTEM, PSP_HOST_NAMESPACE, PSP_HOST_NETWORK_PORTS, PSP_PRIVILEGED, PSP_VOLUME_TYPES]

_POD_MATCH = {"kinds": [{"apiGroups": [""], "kinds": ["Pod"]}]}
PSP_CONSTRAINTS = [
    constraint("K8sPSPHostFilesystem", "psp-host-filesystem", match=_POD_MATCH,
               parameters={"allowedHostPaths": [{"readOnly": True, "pathPrefix": "/foo"}]}),
    constraint("K8sPSPHostNamespace", "psp-host-namespace", match=_POD_MATCH),
    constraint("K8sPSPHostNetworkingPorts", "psp-host-network-ports", match=_POD_MATCH,
               parameters={"hostNetwork": True, "min": 80, "max": 9000}),
    constraint("K8sPSPPrivilegedContainer", "psp-privileged-container", match=_POD_MATCH),
    constraint("K8sPSPVolumeTypes", "psp-volume-types", match=_POD_MATCH,
               parameters={"volumes": ["configMap", "emptyDir", "projected", "secret", "downwardAPI",
                                       "persistentVolumeClaim", "flexVolume"]}),
]


def _psp_pod(name, spec):
    return {"apiVersion": "v1", "kind": "Pod", "metadata": {"name": name, "labels": {"app": name}}, "spec": spec}


PSP_PODS = [
    _psp_pod("nginx-host-filesystem", {
        "containers": [{"name": "nginx", "image": "nginx",
                        "volumeMounts": [{"mountPath": "/cache", "name": "cache-volume", "readOnly": True}]}],
        "volumes": [{"name": "cache-volume", "hostPath": {"path": "/tmp"}}]}),
    _psp_pod("nginx-host-namespace", {"hostPID": True, "hostIPC": True,
                                      "containers": [{"name": "nginx", "image": "nginx"}]}),
    _psp_pod("nginx-host-networking-ports", {
        "hostNetwork": True,
        "containers": [{"name": "nginx", "image": "nginx", "ports": [{"containerPort": 9001, "hostPort": 9001}]}]}),
    _psp_pod("nginx-privileged", {"containers": [{"name": "nginx", "image": "nginx",
                                                  "securityContext": {"privileged": True}}]}),
    _psp_pod("nginx-volume-types", {
        "containers": [{"name": "nginx", "image": "nginx", "volumeMounts": [{"mountPath": "/cache", "name": "cache-volume"}]},
                       {"name": "nginx2", "image": "nginx", "volumeMounts": [{"mountPath": "/cache2", "name": "demo-vol"}]}],
        "volumes": [{"name": "cache-volume", "hostPath": {"path": "/tmp"}}, {"name": "demo-vol", "emptyDir": {}}]}),
]


def config5(load=5, seed=99):
    """The PSP templates with `load` constraints: generateConstraints
    (policy_benchmark_test.go:176-186) cycles through the 5 constraints, every
    copy after the first round under a fresh random 10-letter name."""
    rng = random.Random(seed)
    cs = []
    names = [c["metadata"]["name"] for c in PSP_CONSTRAINTS]
    for i in range(load):
        base = PSP_CONSTRAINTS[i % len(PSP_CONSTRAINTS)]
        c = json.loads(json.dumps(base))
        c["metadata"]["name"] = names[i % len(names)]
        names[i % len(names)] = "".join(rng.choice("abcdefghijklmnopqrstuvwxyz") for _ in range(10))
        cs.append(c)
    return list(PSP_TEMPLATES), cs


def admission_request(n, rng):
    """createAdmissionRequests (policy_benchmark_test.go:197-231): the n-th
    UPDATE request over PSP pod n % 5, object at resourceVersion 2 and
    oldObject at 1, as admission/v1beta1 AdmissionRequest JSON (field order and
    omitempty of k8s.io/api/admission/v1beta1/types.go:45-112)."""
    pod = json.loads(json.dumps(PSP_PODS[n % len(PSP_PODS)]))
    name, namespace = "res-name-%d" % n, "res-namespace-%d" % n
    pod["metadata"]["name"] = name
    pod["metadata"]["namespace"] = namespace
    old = json.loads(json.dumps(pod))
    pod["metadata"]["resourceVersion"] = "2"
    old["metadata"]["resourceVersion"] = "1"
    uid = "%08x-%04x-4%03x-%04x-%012x" % (rng.getrandbits(32), rng.getrandbits(16), rng.getrandbits(12),
                                          0x8000 | rng.getrandbits(14), rng.getrandbits(48))
    gvk = {"group": "", "version": "v1", "kind": "Pod"}
    gvr = {"group": "", "version": "v1", "resource": "pods"}
    return {"uid": uid, "kind": gvk, "resource": gvr, "requestKind": dict(gvk), "requestResource": dict(gvr),
            "name": name, "namespace": namespace, "operation": "UPDATE",
            "userInfo": {"username": "res-creator", "uid": "uid", "groups": ["res-creator-group"],
                         "extra": {"extraKey": ["value1", "value2"]}},
            "object": pod, "oldObject": old, "dryRun": False, "options": None}


def gen_admission_inputs(n, seed=99, start=0):
    """n Query inputs {"review": gkReview} for AugmentedReview{request, ns}
    (policy.go:363-387 with the benchmark's fake namespace getter), JSON text."""
    from .webhook import namespace_object, review_input
    rng = random.Random(seed * 7919 + start)
    out = []
    for i in range(start, start + n):
        req = admission_request(i, rng)
        out.append(dumps(review_input(req, namespace_object(req["namespace"]))))
    return out
