"""Mirror of the frameworks Client calls that reach the driver.

Follows vendor/github.com/open-policy-agent/frameworks/constraint/pkg/client/client.go
(AddTemplate :350-395, AddConstraint :535-577, AddData :91-113, Review :763-800,
Audit :805-833) and the K8s target handler pkg/target/target.go
(ProcessData :62-89, HandleReview / augmentedUnstructuredToAdmissionRequest
:91-163).  The template package rewrite stands in for regorewriter's
AST rewrite (client.go:280-347): the entry module's `package` clause becomes
`templates["<target>"]["<Kind>"]`.
"""
from __future__ import annotations

import json
import re
import urllib.parse
from typing import Optional

TARGET = "admission.k8s.gatekeeper.sh"
CONSTRAINT_GROUP = "constraints.gatekeeper.sh"

# corev1.Namespace{} marshalled by encoding/json (cluster-scoped objects in audit)
EMPTY_NAMESPACE = {"metadata": {"creationTimestamp": None}, "spec": {}, "status": {}}


def template_kind(template: dict) -> str:
    return template["spec"]["crd"]["spec"]["names"]["kind"]


class TemplateError(ValueError):
    """AddTemplate's rejection of a template's Rego (client.go:280-347)."""


# fields under `data` a template may read besides its libs (rego_helpers.go:12-14)
ALLOWED_DATA_FIELDS = ("inventory",)


def _code_spans(src: str):
    """[start, end) spans of src outside string literals and comments"""
    spans, i, start, n = [], 0, 0, len(src)
    while i < n:
        c = src[i]
        if c == '"' or c == "`" or c == "#":
            if i > start:
                spans.append((start, i))
            if c == "#":
                j = src.find("\n", i)
                i = n if j < 0 else j
            elif c == "`":
                j = src.find("`", i + 1)
                i = n if j < 0 else j + 1
            else:
                j = i + 1
                while j < n and src[j] != '"':
                    j += 2 if src[j] == "\\" else 1
                i = min(n, j + 1)
            start = i
            continue
        i += 1
    if start < n:
        spans.append((start, n))
    return spans


_DATA_REF = re.compile(r"(?<![\w.])data((?:\s*\.\s*[A-Za-z_][A-Za-z0-9_]*|\s*\[\s*\"[^\"\\\\]*\"\s*\])*)")
_SEG = re.compile(r"\.\s*([A-Za-z_][A-Za-z0-9_]*)|\[\s*\"([^\"\\\\]*)\"\s*\]")


def _ref_path(tail: str):
    return [a or b for a, b in _SEG.findall(tail)]


def _rewrite_module(src: str, lib_prefix, is_lib: bool):
    """regorewriter.Rewrite (regorewriter.go:366-419) over one module's text:
    checks every `data` ref (a lib or an allowed extern, :250-271) and every
    import (:274-291), prefixes `data.lib...` refs and imports with lib_prefix
    (PackagePrefixer.Transform, packagetransformer.go:32-40), and for a lib
    moves its `package lib.<x>` under the prefix (:371-373; the package must
    be strictly below `lib`, :224-247)."""
    out, pos = [], 0
    pkg_done = False
    for a, b in _code_spans(src):
        out.append(src[pos:a])
        seg = src[a:b]
        res, p = [], 0
        if not pkg_done:
            m = re.search(r"(?m)^\s*package\s+([A-Za-z_][\w.]*)", seg)
            if m:
                pkg_done = True
                if is_lib:
                    path = m.group(1).split(".")
                    if path[0] != "lib" or len(path) < 2:
                        raise TemplateError("path data.%s not found in lib prefixes" % m.group(1))
                    res.append(seg[:m.start(1)] + ".".join(lib_prefix + path))
                    p = m.end(1)
        for m in re.finditer(r"(?m)^\s*import\s+([A-Za-z_][\w.\[\]\"]*)", seg[p:]):
            imp = m.group(1)
            if not (imp == "data.lib" or imp.startswith("data.lib.") or imp.startswith('data["lib"]')):
                raise TemplateError("bad import")
        for m in _DATA_REF.finditer(seg, p):
            path = _ref_path(m.group(1))
            if not path:
                continue  # bare `data`: checkRef finds no rule to reject (a local use of the whole tree)
            if path[0] in ALLOWED_DATA_FIELDS:
                continue
            if path[0] != "lib":
                raise TemplateError("disallowed ref data.%s" % ".".join(path))
            res.append(seg[p:m.start()] + "data." + ".".join(lib_prefix + path))
            p = m.end()
        res.append(seg[p:])
        out.append("".join(res))
        pos = b
    out.append(src[pos:])
    return "".join(out)


def template_modules(template: dict):
    """(prefix, [entry module, libs...]) as createTemplateArtifacts builds them
    (client.go:280-347): the entry module's package becomes
    `templates["<target>"]["<Kind>"]`, and the libs and every `data.lib` ref
    move under `libs.<target>.<Kind>` (templateLibPrefix, client.go:147-150),
    so two templates' libs never collide.  Raises TemplateError where
    regorewriter rejects the sources."""
    kind = template_kind(template)
    tgt = template["spec"]["targets"][0]
    src = tgt["rego"]
    prefix = 'templates["%s"]["%s"]' % (TARGET, kind)
    lib_prefix = ("libs.%s.%s" % (TARGET, kind)).split(".")
    src = re.sub(r"^\s*package\s+\S+", "package " + prefix, src, count=1, flags=re.M)
    mods = [_rewrite_module(src, lib_prefix, False)]
    for lib in tgt.get("libs", []) or []:
        mods.append(_rewrite_module(lib, lib_prefix, True))
    return prefix, mods


def constraint_path(constraint: dict) -> str:
    return "/constraints/%s/cluster/%s/%s/%s" % (TARGET, CONSTRAINT_GROUP, constraint["kind"], constraint["metadata"]["name"])


def group_version(api_version: str):
    """schema.ParseGroupVersion (k8s.io/apimachinery schema/group_version.go):
    "" and "/" -> ("", ""), "v" -> ("", v), "g/v" -> (g, v); more slashes are
    an error, which unstructured.GroupVersionKind turns into an EMPTY GVK
    (unstructured.go:425-432) -- kind included, see gvk_of"""
    if "/" not in api_version:
        return "", api_version
    parts = api_version.split("/")
    if len(parts) == 2:
        return parts[0], parts[1]
    return "", ""


def gvk_of(obj: dict):
    """obj.GroupVersionKind() (unstructured.go:425-432): (group, version, kind),
    all empty when apiVersion does not parse"""
    av = obj.get("apiVersion", "") if isinstance(obj.get("apiVersion"), str) else ""
    kind = obj.get("kind", "") if isinstance(obj.get("kind"), str) else ""
    if av.count("/") > 1:
        return "", "", ""
    g, v = group_version(av)
    return g, v, kind


def data_path(obj: dict) -> str:
    """K8sValidationTarget.ProcessData (target.go:62-76)."""
    gv = obj.get("apiVersion", "")
    kind = obj.get("kind", "")
    name = obj.get("metadata", {}).get("name", "")
    ns = obj.get("metadata", {}).get("namespace", "")
    esc = urllib.parse.quote(gv, safe="")
    if not ns:
        return "/external/%s/cluster/%s/%s/%s" % (TARGET, esc, kind, name)
    return "/external/%s/namespace/%s/%s/%s/%s" % (TARGET, ns, esc, kind, name)


def augmented_review(obj: dict, ns: Optional[dict]) -> dict:
    """gkReview JSON for Review(AugmentedUnstructured{obj, ns}) (target.go:129-163):
    admission/v1beta1 AdmissionRequest field order, omitempty name/namespace."""
    group, version, kind = gvk_of(obj)
    md = obj.get("metadata") if isinstance(obj.get("metadata"), dict) else {}
    name = md.get("name", "") if isinstance(md.get("name"), str) else ""
    nsobj = ns if ns is not None else EMPTY_NAMESPACE
    nsmd = nsobj.get("metadata") if isinstance(nsobj.get("metadata"), dict) else {}
    nsname = nsmd.get("name", "") if isinstance(nsmd.get("name"), str) else ""
    r = {"uid": "", "kind": {"group": group, "version": version, "kind": kind},
         "resource": {"group": "", "version": "", "resource": ""}}
    if name:
        r["name"] = name
    if nsname:
        r["namespace"] = nsname
    r.update({"operation": "", "userInfo": {}, "object": obj, "oldObject": None, "options": None,
              "_unstable": {"namespace": nsobj}})
    return r


class Client:
    """The driver-facing half of frameworks client.Client for the K8s target."""

    def __init__(self, driver):
        self.driver = driver
        # Client.init (client.go:667-722): target hooks + match library modules.
        # The engine serves both natively; their packages are what it keys on.
        driver.put_module('hooks["%s"].hooks_builtin' % TARGET, 'package hooks["%s"]\n' % TARGET)
        driver.put_module('hooks["%s"].library' % TARGET, 'package hooks["%s"].library\n' % TARGET)
        driver.init()

    def add_template(self, template: dict):
        prefix, mods = template_modules(template)
        self.driver.put_modules(prefix, mods)
        return template_kind(template)

    def remove_template(self, template: dict):
        prefix, _ = template_modules(template)
        return self.driver.delete_modules(prefix)

    def add_constraint(self, constraint: dict):
        self.driver.put_data(constraint_path(constraint), constraint)

    def remove_constraint(self, constraint: dict):
        return self.driver.delete_data(constraint_path(constraint))

    def add_data(self, obj: dict):
        self.driver.put_data(data_path(obj), obj)

    def remove_data(self, obj: dict):
        return self.driver.delete_data(data_path(obj))

    def review(self, review: dict):
        """Client.Review (client.go:763-800): Driver.Query, then HandleViolation
        (target.go:193-244) on every result; its error fails the Review."""
        from .target import handle_violation
        res = self.driver.query('hooks["%s"].violation' % TARGET, {"review": review})
        if res.results:
            resource = handle_violation(review)
            for r in res.results:
                r.resource = resource
        return res

    def review_objects(self, objs, namespaces):
        return self.driver.review_objects(objs, namespaces)

    def audit(self):
        return self.driver.query('hooks["%s"].audit' % TARGET, None)

    def reset(self):
        self.driver.delete_data("/external/%s" % TARGET)
        self.driver.delete_data("/constraints/%s" % TARGET)
