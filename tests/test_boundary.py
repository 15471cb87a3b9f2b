"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports
every symbol include/gkgpu.h declares, templates compile (or are explicitly
marked for CPU fallback), driver bookkeeping mirrors drivers.Driver."""
import os
import re

import pytest

import gkgpu
from gkgpu import workloads as W
from gkgpu.client import Client, template_modules

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gkgpu.h")


def header_symbols():
    txt = open(HEADER).read()
    decl = r"^\s*(?:int|void|const char\s*\*|size_t|uint32_t|uint64_t)\s+\**(gk_\w+)\s*\("
    return sorted(set(re.findall(decl, txt, re.M)))


def test_library_exports_every_header_symbol():
    lib = gkgpu.load_library()
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(gkgpu.driver.EXPORTS) <= set(syms)


def test_subset_templates_compile_to_gpu_bytecode():
    d = gkgpu.Driver()
    cl = Client(d)
    for t in [W.REQUIRED_LABELS_BASIC, W.REQUIRED_LABELS, W.ALLOWED_REPOS, W.CONTAINER_LIMITS, W.REQUIRED_PROBES,
              W.ALLOWED_LABEL_REGEX, W.ALLOWED_ANNOTATION_REGEX]:
        kind = cl.add_template(t)
        st, why = d.template_status(kind)
        assert st == 1, (kind, why)


GUARDED = W._tmpl("K8sGuardedEncode", """package k8sguardedencode

violation[{"msg": msg}] {
	input.review.kind.kind == "Service"
	input.review.kind.version == "v1"
	input.review.kind.group == ""
	x := base64.encode(input.review.object.metadata.name)
	msg := sprintf("encoded <%v>", [x])
}
""")


def test_out_of_subset_template_is_explicit_fallback():
    d = gkgpu.Driver()
    cl = Client(d)
    t = W._tmpl("K8sEncode", """package k8sencode

violation[{"msg": msg}] {
	x := base64.encode(input.review.object.metadata.name)
	msg := sprintf("encoded <%v>", [x])
}
""")
    kind = cl.add_template(t)
    st, why = d.template_status(kind)
    assert st == 0 and "base64.encode" in why
    # the guard program: no expression before the builtin, so every matched review falls back
    b, why2 = d.template_backend(kind)
    assert b == 3 and "base64.encode" in why2


def test_guard_program_evaluates_the_supported_prefix():
    """A template outside the subset (an unsupported builtin) compiles into a
    device guard: its `input.review.kind` tests run ahead of the first
    unsupported expression, which is the only fallback point."""
    d = gkgpu.Driver(jit=False)
    cl = Client(d)
    kind = cl.add_template(GUARDED)
    st, why = d.template_status(kind)
    assert st == 0 and "base64.encode" in why
    b, _ = d.template_backend(kind)
    assert b == 3
    asm = d.debug_disasm(kind)
    assert asm.count("FAIL_FALLBACK") >= 1
    # the guard compares kind, version and group before the first fallback point
    head = asm[:asm.index("FAIL_FALLBACK")]
    for lit in ('"Service"', '"v1"', '""'):
        assert lit in head


def test_unique_service_selector_join_compiles_to_the_gpu_subset():
    """demo/agilebank's unique-service-selector (sort + the data.inventory join,
    regolib src.go:30-31,66-72) is inside the subset: data.inventory is a
    constant document node the engine points at the synced inventory tree."""
    for jit in (False, True):
        d = gkgpu.Driver(jit=jit)
        cl = Client(d)
        kind = cl.add_template(W.UNIQUE_SERVICE_SELECTOR)
        st, why = d.template_status(kind)
        assert st == 1, why
        b, detail = d.template_backend(kind)
        assert b == (2 if jit else 1), detail
    asm = gkgpu.Driver(jit=False)
    cl = Client(asm)
    cl.add_template(W.UNIQUE_SERVICE_SELECTOR)
    text = asm.debug_disasm("K8sUniqueServiceSelector")
    assert "FAIL_FALLBACK" not in text
    assert "sort" in text or "CALL" in text


def test_put_modules_replaces_and_delete_modules_counts():
    d = gkgpu.Driver()
    prefix, mods = template_modules(W.ALLOWED_REPOS)
    d.put_modules(prefix, mods)
    d.put_modules(prefix, mods)
    assert d.delete_modules(prefix) == 1
    assert d.delete_modules(prefix) == 0


def test_bad_rego_is_a_put_error():
    d = gkgpu.Driver()
    with pytest.raises(RuntimeError):
        d.put_module("x", "package p\n\nviolation[{\"msg\": msg}] {\n\tmsg := \n}\n")


def test_constraints_and_delete_data():
    d = gkgpu.Driver()
    cl = Client(d)
    ts, cs = W.config2()
    for t in ts:
        cl.add_template(t)
    for c in cs:
        cl.add_constraint(c)
    assert len(d.constraints()) == 5
    assert cl.remove_constraint(cs[0]) is True
    assert len(d.constraints()) == 4
    cl.reset()
    assert d.constraints() == []


def test_dump_lists_modules():
    d = gkgpu.Driver()
    cl = Client(d)
    cl.add_template(W.REQUIRED_LABELS_BASIC)
    s = d.dump()
    assert "K8sRequiredLabels" in s


def test_compressed_regex_dfa_agrees_with_the_full_table():
    """regex.cc compress_regex_dfa (the byte-class form a wavefront stages in
    LDS, devrt.h re_run_lds) decides every subject exactly as the full
    129-word-per-state table does (run_regex_dfa / devrt.h re_run)."""
    import ctypes
    import random
    lib = gkgpu.load_library()
    full, comp = lib.gk_regex_test, lib.gk_regex_ctest
    for f in (full, comp):
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
    pats = ["^[a-z]+$", "^prod-[0-9]{2,4}$", "^(dev|staging|prod)$", "^[0-9]+$", "a|b|c", "^$", "x*y+",
            "^[A-Za-z0-9_.-]{1,63}$", "team-[a-f0-9]+", "^https?://", "é+", "^v[0-9]+\\.[0-9]+(\\.[0-9]+)?$"]
    rng = random.Random(3)
    alphabet = b"abcxyz019-_.:/prodevstagingAZ\xc3\xa9 "
    seen_match = 0
    for p in pats:
        subjects = [b"", b"prod", b"prod-12", b"staging", b"v1.2.3", b"https://x", b"\xc3\xa9\xc3\xa9", b"team-ab12"]
        subjects += [bytes(rng.choice(alphabet) for _ in range(rng.randrange(0, 16))) for _ in range(300)]
        for s in subjects:
            a = full(p.encode(), s, len(s))
            b = comp(p.encode(), s, len(s))
            if b == -3:
                continue  # does not compress: the device walks the full table
            assert a == b, (p, s, a, b)
            seen_match += a == 1
    assert seen_match > 50
