"""The canonical message comparator (tests/canonical.py): the Go-map order of
printed objects (ast/term.go:79-92) is not compared; everything else is."""
from canonical import canonical_message


def test_object_member_order_is_not_compared():
    a = 'bad parameters: {"hostNetwork": false, "ranges": [{"max": 9000, "min": 80}]}'
    b = 'bad parameters: {"ranges": [{"min": 80, "max": 9000}], "hostNetwork": false}'
    assert canonical_message(a) == canonical_message(b)
    assert canonical_message(a) != canonical_message(a.replace("9000", "9001"))


def test_sets_plain_text_and_arrays():
    assert canonical_message('you must provide labels: {"b", "a"}') == \
        canonical_message('you must provide labels: {"a", "b"}')
    # array order is significant
    assert canonical_message("x [1, 2]") != canonical_message("x [2, 1]")
    assert canonical_message("set() and {} and {oops") == "set() and {} and {oops"
    plain = "container <nginx> has no resource limits"
    assert canonical_message(plain) == plain


def test_nested_and_quoted_braces():
    m = 'v {"a": {"z": "}", "y": "{"}, "b": set()}'
    n = 'v {"b": set(), "a": {"y": "{", "z": "}"}}'
    assert canonical_message(m) == canonical_message(n)


def test_parity_compares_deterministic_sets_byte_for_byte():
    """tests/parity.py rows_agree: a set built from an array prints in array
    order in the reference (k8srequiredlabels' `missing`,
    demo/agilebank/templates/k8srequiredlabels_template.yaml:39-46), so a
    different member order is a mismatch; only the object-printing PSP
    templates compare canonically."""
    from parity import rows_agree
    row = lambda kind, msg: (kind, "c", msg, "{}", "deny")
    want = [row("K8sRequiredLabels", 'you must provide labels: {"a", "b"}')]
    got = [row("K8sRequiredLabels", 'you must provide labels: {"b", "a"}')]
    assert rows_agree(want, want) == "exact"
    assert rows_agree(want, got) is None
    pw = [row("K8sPSPHostNetworkingPorts", 'Allowed values: {"hostNetwork": false, "max": 9}')]
    pg = [row("K8sPSPHostNetworkingPorts", 'Allowed values: {"max": 9, "hostNetwork": false}')]
    assert rows_agree(pw, pg) == "canonical"
    # a mixed review: the PSP row may differ in member order, the other may not
    assert rows_agree(want + pw, want + pg) == "canonical"
    assert rows_agree(want + pw, got + pg) is None
