"""Fixtures from the reference's bats e2e suite (test/bats/): the
K8sContainerLimits template whose helpers live in a template lib
(tests/templates/k8scontainterlimits_template.yaml: `libs:` + `import
data.lib.helpers`), its constraint, and the two Pods test.bats:130-134 applies
with their expected admission outcome (opa_no_limits denied, opa allowed).

Run in the build container (reads /root/reference, writes bats_fixtures.json);
the JSON is the committed data the tests use.
"""
import json
import os

import yaml

REF = "/root/reference/test/bats"
HERE = os.path.dirname(os.path.abspath(__file__))


def load(rel):
    with open(os.path.join(REF, rel)) as f:
        return yaml.safe_load(f)


def main():
    out = {
        "source": "test/bats/tests (templates/k8scontainterlimits_template.yaml, "
                  "constraints/containers_must_be_limited.yaml, bad/opa_no_limits.yaml, good/opa.yaml); "
                  "outcomes from test/bats/test.bats:130-134",
        "template": load("tests/templates/k8scontainterlimits_template.yaml"),
        "constraint": load("tests/constraints/containers_must_be_limited.yaml"),
        "pods": [
            {"object": load("tests/bad/opa_no_limits.yaml"), "namespace": "good-ns", "denied": True},
            {"object": load("tests/good/opa.yaml"), "namespace": "good-ns", "denied": False},
        ],
    }
    with open(os.path.join(HERE, "bats_fixtures.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
