"""The match-library KATs replayed through the engine's device runtime built
for the host (oracle/cpuvm.cc runs devrt.h's match stage and the template
bytecode on CPU threads): the same triples tests/test_gpu_parity.py replays on
the MI355X, checked here on every CPU run.  Counts only: a violation per
matched deny-all constraint, one per autoreject, flagged pairs for errors."""
import pytest

import gkgpu
from kat_replay import cases, engine_for, expected, query_input

CASES = cases()


def test_replay_covers_match_functions():
    fns = {c["fn"] for c in CASES}
    assert len(CASES) >= 100 and len(fns) == 8


@pytest.mark.parametrize("case", CASES, ids=[c["id"] for c in CASES])
def test_kat_on_host_device_runtime(case):
    from oracle import cpu_baseline as CB
    want = expected(case)
    drv = gkgpu.Driver(jit=False, host_only=True)
    engine_for(drv, case)
    b = drv.debug_stage_inputs([query_input(case)])
    _s, evals, viol, _mb, flagged = CB.sweep(drv, b, threads=1)
    if want == "ERROR":
        assert flagged > 0
    else:
        assert flagged == 0
        assert viol == len(want), (case["id"], want)
