"""re_match as Go's regexp decides it (OPA v0.21 topdown/regex.go:21-34:
regexp.Compile + an unanchored match over the UTF-8 text), in the engine's DFA
compiler (gatekeeper-1_amd/csrc/regex.cc, the tables every kernel walks) and in
the oracle's translation onto Python `re` (oracle/rego/goregex.py).

Parity UNPINNED: the reference holds no regex vectors.  The
known answers below restate Go's documented syntax (regexp/syntax):
  * `\\s` is the Perl class [\\t\\n\\f\\r ] -- no \\v (Python's ASCII \\s has it);
  * (?i) is simple case folding (unicode.SimpleFold): k/K/U+212A (KELVIN SIGN)
    and s/S/U+017F (LATIN SMALL LETTER LONG S) are orbits, i/I is not paired
    with U+0130/U+0131; Perl classes and bracket classes fold too;
  * flags set mid-group hold to the end of that group.
The engine may answer -2 (CPU fallback) where its DFA is utf8-sensitive and
the subject is not ASCII; every other answer must equal the oracle's."""
import ctypes
import random

import pytest

import gkgpu
from oracle.rego.goregex import re_match
from oracle.rego.values import RegoError

KELVIN, LONG_S = "\u212a", "\u017f"

# (pattern, subject, Go's answer)
KATS = [
    (r"^\s$", "\v", False),
    (r"^\s$", " ", True),
    (r"^\s$", "\t", True),
    (r"^\s$", "\x0c", True),
    (r"^[\s]$", "\v", False),
    (r"^\S$", "\v", True),
    (r"^\v$", "\v", True),
    (r"(?i)^k$", KELVIN, True),
    (r"(?i)^K$", KELVIN, True),
    (r"(?i)^k$", "K", True),
    (r"^k$", KELVIN, False),
    (r"(?i)^s$", LONG_S, True),
    (r"(?i)^S+$", "s" + LONG_S + "S", True),
    (r"(?i)^i$", "\u0130", False),
    (r"(?i)^i$", "\u0131", False),
    (r"(?i)^[a-z]+$", KELVIN + LONG_S + "x", True),
    (r"^[a-z]+$", KELVIN, False),
    (r"(?i)^\w$", KELVIN, True),
    (r"(?i)^[^k]$", KELVIN, False),
    (r"(?i)^[^a]$", KELVIN, True),
    (r"a(?i)b", "aB", True),
    (r"a(?i)b", "AB", False),
    (r"(a(?i)b)c", "aBC", False),
    (r"(a(?i)b)c", "aBc", True),
    (r"(?i:k)k", KELVIN + "k", True),
    (r"(?i:k)k", "k" + KELVIN, False),
    (r"(?i)a(?-i)k", "AK", False),
    (r"(?i)a(?-i)k", "Ak", True),
    (r"^[a-z]+.agilebank.demo$", "ops.agilebank.demo\n", False),
    (r"^(dev|stage|prod)-[0-9]{1,4}$", "prod-12", True),
]


def _engine():
    lib = gkgpu.load_library()
    f = lib.gk_regex_test
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    return lambda p, s: f(p.encode(), s.encode(), len(s.encode()))


@pytest.mark.parametrize("pat,subj,want", KATS)
def test_go_regex_known_answers(pat, subj, want):
    assert re_match(pat, subj) is want, ("oracle", pat, subj)
    got = _engine()(pat, subj)
    assert got in (int(want), -2), ("engine", pat, subj, got)
    if subj.isascii():
        assert got == int(want), ("engine decides ASCII subjects", pat, subj, got)


def test_kelvin_and_long_s_are_decided_on_the_device_tables():
    """the fold partners are byte sequences of the DFA, not a fallback"""
    eng = _engine()
    assert eng(r"(?i)^k$", KELVIN) == 1
    assert eng(r"(?i)^[a-z]+$", "o" + LONG_S) == 1
    assert eng(r"(?i)^[a-z]+$", "o\u0130") == 0


PATTERNS = [r"^[a-zA-Z]+.agilebank.demo$", r"^(dev|stage|prod)-[0-9]{1,4}$", r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$",
            r"(?i)^team-[a-z]+$", r"(?i)k+s", r"\s", r"^\S+$", r"[\s,]+", r"(?i)\w+$", r"^[^\s]+$",
            r"(?i)^(ks|sk)$", r"x(?i)k|s", r"(?i:[k-s])+z", r"^\d{2}\s\w+$", r"(?i)[^s]k"]
ALPHABET = ["a", "k", "K", "s", "S", "z", "x", "-", "0", "7", " ", "\t", "\v", "\n", ",", ".", KELVIN, LONG_S,
            "\u0130", "\u00e9", "team", "prod", "dev", "agilebank", "demo"]


def test_engine_agrees_with_oracle_on_random_subjects():
    eng = _engine()
    rng = random.Random(11)
    decided = matched = 0
    for p in PATTERNS:
        subjects = ["", "ks", KELVIN + LONG_S, "team-" + KELVIN, "prod-12", "ops.agilebank.demo", "12 ab"]
        subjects += ["".join(rng.choice(ALPHABET) for _ in range(rng.randrange(0, 7))) for _ in range(250)]
        for s in subjects:
            try:
                want = re_match(p, s)
            except (RegoError, NotImplementedError):
                continue
            got = eng(p, s)
            if got == -2:
                assert not s.isascii(), (p, s)
                continue
            assert got == int(want), (p, s, got, want)
            decided += 1
            matched += got
    assert decided > 2500 and matched > 300, (decided, matched)
