"""Generate tests/golden/match_kats.jsonl from the reference's own Rego KATs.

Run HERE (needs /root/reference; never on the GPU box):
    python tests/golden/gen_match_kats.py

For every `test_*` rule in pkg/target/regolib/*_test.rego the reference's
library (pkg/target/regolib/src.rego) and the test module are loaded into the
oracle interpreter (oracle.rego); the test must pass (all 109 do), and every
library call made directly from the test body is recorded as a golden vector:
(function, argument values, input, data, result).  The reference Rego text is
only read here; the fixture holds values, not source.
"""
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.codec import enc  # noqa: E402
from oracle.match import UNDEF  # noqa: E402
from oracle.rego import Interpreter  # noqa: E402
from oracle.rego.interp import _UNDEF  # noqa: E402

REF = "/root/reference/pkg/target/regolib"
CROOT = "{{.ConstraintsRoot}}"
DROOT = "{{.DataRoot}}"
RECORD = {"matches_label_selector", "any_labelselector_match", "any_kind_selector_matches", "matches_scope",
          "matches_namespaces", "does_not_match_excludednamespaces", "matches_nsselector", "has_field",
          "get_default", "make_group_version"}


class Recorder(Interpreter):
    def __init__(self):
        super().__init__()
        self.depth = 0
        self.records = []
        self.cur_test = None

    def _call_func(self, rules, vals, statement, ctx):
        name = rules[0].name
        rec = self.depth == 0 and name in RECORD and rules[0].package == ("target",)
        self.depth += 1
        got = []
        try:
            for v in super()._call_func(rules, vals, statement, ctx):
                got.append(v)
        finally:
            self.depth -= 1
        if rec:
            self._record(name, vals, got[0] if got else UNDEF, ctx, statement)
        for v in got:
            yield v

    def eval_rule_ref(self, rules, path, i, b, env):
        name = rules[0].name
        rec = self.depth == 0 and name == "autoreject_review" and i == len(path)
        inc = 0 if name.startswith("test_") else 1
        self.depth += inc
        try:
            out = list(super().eval_rule_ref(rules, path, i, b, env))
        finally:
            self.depth -= inc
        if rec:
            self._record(name, [], out[0][0] if out else UNDEF, env.ctx, False)
        for x in out:
            yield x

    def _record(self, name, vals, result, ctx, statement):
        inp = ctx.input if ctx.input is not _UNDEF else UNDEF
        data = ctx.data
        croot = data.get(CROOT) if CROOT in data else UNDEF
        ext = data.get(DROOT) if DROOT in data else UNDEF
        self.records.append({
            "test": self.cur_test, "fn": name, "args": [enc(v) for v in vals], "input": enc(inp),
            "constraints": enc(croot), "external": enc(ext), "statement": statement, "result": enc(result),
        })


def main():
    it = Recorder()
    it.add_module(open(os.path.join(REF, "src.rego")).read())
    tests = []
    for f in sorted(glob.glob(os.path.join(REF, "*_test.rego"))):
        m = it.add_module(open(f).read())
        tests += [(os.path.basename(f), r.name) for r in m.rules if r.name.startswith("test_")]
    failed = []
    for f, name in tests:
        it.cur_test = "%s:%s" % (f, name)
        if not it.run_test_rule(("target",), name):
            failed.append(it.cur_test)
    assert not failed, failed
    out = os.path.join(HERE, "match_kats.jsonl")
    with open(out, "w") as fh:
        for r in it.records:
            fh.write(json.dumps(r, sort_keys=True) + "\n")
    print("tests passed: %d, vectors: %d -> %s" % (len(tests), len(it.records), out))


if __name__ == "__main__":
    main()
