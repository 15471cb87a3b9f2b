"""CPU oracle for the Gatekeeper audit hot path — TEST INFRASTRUCTURE ONLY.

This package is a from-scratch Python restatement of the reference's evaluation
semantics (OPA v0.21 topdown + the frameworks hooks + the pkg/target match
library).  It exists to check the MI355X engine; only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The product path (``gatekeeper-1_amd/``) never imports or calls it.

Pinning: ``tests/golden/gen_match_kats.py`` runs the reference's own
``pkg/target/regolib/*_test.rego`` known-answer tests (109 cases) through
``oracle.rego`` and records every library call as a golden vector; the
restated match library (``oracle.match``) is checked against those vectors.
Regex (Go RE2) and float formatting are "parity unpinned" — the reference holds
no test for them.
"""
