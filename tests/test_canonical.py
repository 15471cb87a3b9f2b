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
