"""k_feasibility (the static pod-state x instance-type rows): k_solve with the rows ANDed in
(the default whenever a pod carries label requirements) and with every key evaluated per step
(KS_NO_FEASIBILITY, read at ks_problem_create) return the same Results, and both equal the oracle.
The rows factor Requirements.Intersects over single-valued keys (requirements.go:241-258); these problems
carry In / NotIn / Exists / DoesNotExist / Gt / Lt terms, OR'd node-affinity terms, preferred terms and
multi-zone offerings, so both factors and the multi-valued remainder are exercised."""
import json
import os

import pytest

import problems
from karpenter_amd import Scheduler, synth
from oracle import bridge

pytestmark = pytest.mark.gpu


def _solve(snap_json, rows):
    if rows:
        os.environ.pop("KS_NO_FEASIBILITY", None)
    else:
        os.environ["KS_NO_FEASIBILITY"] = "1"
    try:
        sch = Scheduler(snap_json)
        r = sch.solve()
        sch.close()
        return r
    finally:
        os.environ.pop("KS_NO_FEASIBILITY", None)


CASES = [("random", s) for s in range(8)] + [("special", s) for s in range(20, 36)] + [("c3", 1500)]


@pytest.mark.parametrize("kind,arg", CASES, ids=["%s-%s" % c for c in CASES])
def test_feasibility_rows_change_nothing(kind, arg):
    """special: NodePool and pod terms on the key some instance types hold as DoesNotExist, where a
    template's Exists meets a pod's NotIn (the row passes DoesNotExist positions; k_solve tests them
    against the whole record's operator)."""
    if kind == "c3":
        snap = synth.config3(arg)
    else:
        snap = problems.random_problem(arg, special=kind == "special")
    s = json.dumps(snap)
    with_rows = _solve(s, True)
    without = _solve(s, False)
    assert with_rows.canonical() == without.canonical()
    want, _ = bridge.solve(s)
    assert problems.canonical(want) == with_rows.canonical()
    if kind == "c3":  # the C3 shape has pods with label requirements: the kernel ran and was timed
        assert with_rows.feasibility_ms > 0 and with_rows.feasibility_bytes > 0
        assert without.feasibility_ms == 0
