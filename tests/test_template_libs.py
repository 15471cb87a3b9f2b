"""Template libs (ConstraintTemplate spec.targets[].libs): the regorewriter
rewrite the frameworks Client applies before the driver sees the modules
(client.go:280-347, regorewriter.go:366-419), and the rewritten template
evaluated by the oracle and by the engine's device runtime built for the host.

Fixtures: the reference's e2e deny-all-with-lib template (client/e2e_tests.go:
83-101, restated inline: three lines of Rego) and the bats K8sContainerLimits
template whose helpers are a lib (tests/golden/bats_fixtures.json, made by
tests/golden/gen_bats_fixtures.py)."""
import json
import os

import pytest

import gkgpu
from gkgpu import workloads as W
from gkgpu.client import TARGET, TemplateError, augmented_review, template_modules
from parity import engine_for, oracle_for, oracle_review

HERE = os.path.dirname(os.path.abspath(__file__))
BATS = json.load(open(os.path.join(HERE, "golden", "bats_fixtures.json")))
LIBP = "libs.%s.Foo" % TARGET

DENY_WITH_LIB = ('package foo\n\nimport data.lib.bar\n\nviolation[{"msg": "DENIED", "details": {}}] {\n'
                 '  bar.always[x]\n\tx == "always"\n}')
DENY_LIB = 'package lib.bar\nalways[y] {\n  y = "always"\n}\n'


def _foo(rego, libs=()):
    t = W._tmpl("Foo", rego)
    t["spec"]["targets"][0]["libs"] = list(libs)
    return t


def _constraint(kind, name="ph"):
    return {"apiVersion": "constraints.gatekeeper.sh/v1beta1", "kind": kind, "metadata": {"name": name},
            "spec": {}}


def test_rewrite_moves_libs_under_the_template_prefix():
    prefix, mods = template_modules(_foo(DENY_WITH_LIB, [DENY_LIB]))
    assert prefix == 'templates["%s"]["Foo"]' % TARGET
    assert mods[0].startswith("package " + prefix)
    assert "import data.%s.lib.bar\n" % LIBP in mods[0]
    assert mods[1].startswith("package %s.lib.bar\n" % LIBP)


def test_rewrite_leaves_strings_comments_and_externs():
    rego = ('package foo\nimport data.lib.x\nviolation[{"msg": m}] {\n  # data.lib.y in a comment\n'
            '  m := "data.lib.z"\n  data.inventory.cluster[_]\n  data.lib.x.f(1)\n}')
    _p, mods = template_modules(_foo(rego, ["package lib.x\nf(a) = a { true }\n"]))
    assert "# data.lib.y in a comment" in mods[0] and '"data.lib.z"' in mods[0]
    assert "data.inventory.cluster" in mods[0]
    assert "data.%s.lib.x.f(1)" % LIBP in mods[0]


@pytest.mark.parametrize("rego,libs,why", [
    ("package foo\nviolation[{\"msg\": \"x\"}] { data.other.x }", [], "disallowed ref"),
    ("package foo\nimport input.review\nviolation[{\"msg\": \"x\"}] { true }", [], "bad import"),
    ("package foo\nimport data.inventory\nviolation[{\"msg\": \"x\"}] { true }", [], "bad import"),
    ("package foo\nviolation[{\"msg\": \"x\"}] { true }", ["package lib\nf = 1 { true }"], "lib prefixes"),
    ("package foo\nviolation[{\"msg\": \"x\"}] { true }", ["package helpers\nf = 1 { true }"], "lib prefixes"),
])
def test_rewrite_rejects_what_regorewriter_rejects(rego, libs, why):
    """regorewriter.go checkLibPackages :224-247, checkImport :274-291,
    checkRef :250-271"""
    with pytest.raises(TemplateError, match=why):
        template_modules(_foo(rego, libs))


def test_oracle_deny_all_with_lib():
    """e2e_tests.go 'Deny All With Lib': one DENIED result, enforcementAction deny"""
    od = oracle_for([_foo(DENY_WITH_LIB, [DENY_LIB])], [_constraint("Foo")])
    rows = oracle_review(od, {"kind": {"group": "", "version": "v1", "kind": "Pod"}, "object": {}})
    assert rows == [("Foo", "ph", "DENIED", "{}", "deny")]


def _bats_inputs():
    objs = [p["object"] for p in BATS["pods"]]
    nss = [{"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": p["namespace"]}} for p in BATS["pods"]]
    return objs, nss


def test_oracle_bats_container_limits_outcomes():
    """test.bats:130-134: opa_no_limits is denied, opa (100m / 30Mi) allowed"""
    od = oracle_for([BATS["template"]], [BATS["constraint"]])
    objs, nss = _bats_inputs()
    for p, o, n in zip(BATS["pods"], objs, nss):
        rows = oracle_review(od, augmented_review(o, n))
        assert bool(rows) == p["denied"], rows
    bad = oracle_review(od, augmented_review(objs[0], nss[0]))
    # two bodies (no `resources`, no `resources.limits`) emit the same message;
    # topdown does not dedupe a partial set's values here (eval.go evalOneRule)
    assert [r[2] for r in bad] == ["container <opa> has no resource limits"] * 2


def test_engine_compiles_the_lib_template_on_the_host_runtime():
    """the bats template's lib functions compile into the template program
    (no CPU fallback), and the host build of the device runtime agrees with
    the oracle in counts and message bytes over config 2's Pods"""
    from oracle import cpu_baseline as CB
    drv = gkgpu.Driver(jit=False, host_only=True)
    engine_for(drv, [BATS["template"]], [BATS["constraint"]])
    b, detail = drv.template_backend("K8sContainerLimits")
    assert b in (1, 2), detail
    pods, ns_of, ns_objs = W.gen_pods(600, seed=77, n_namespaces=10)
    objs, nss = _bats_inputs()
    objs = objs + pods
    nss = nss + [ns_objs[n] for n in ns_of]
    batch = drv.stage_objects(objs, nss)
    _s, evals, viol, mbytes, flagged = CB.sweep(drv, batch, threads=2)
    od = oracle_for([BATS["template"]], [BATS["constraint"]])
    want = [oracle_review(od, augmented_review(o, n)) for o, n in zip(objs, nss)]
    assert flagged == 0 and evals == len(objs)
    assert viol == sum(len(w) for w in want) and viol > 100
    assert mbytes == sum(len(r[2].encode()) for w in want for r in w)  # message bytes (details not counted)
