"""Empty and ragged inputs through the GPU path (tests/edge_cases.py): Solve and consolidation results
equal the oracle's exactly, including the reference's quirks (a pod with no template and no node gets
no error, scheduler.go:285; a pass with no candidates simulates nothing)."""
import json

import pytest

import edge_cases
from karpenter_amd import Consolidator
from oracle import bridge
from test_cons_gpu import _first_diff
from test_solve_gpu import _diff, _solve_both

pytestmark = pytest.mark.gpu

SOLVE = edge_cases.solve_cases()
CONS = edge_cases.cons_cases()


@pytest.mark.parametrize("name", sorted(SOLVE))
def test_solve_edge_inputs_parity(name):
    want, got = _solve_both(SOLVE[name])
    assert _diff(want, got) is None, _diff(want, got)


@pytest.mark.parametrize("name", sorted(CONS))
def test_consolidation_edge_inputs_parity(name):
    s = json.dumps(CONS[name])
    want, _ = bridge.consolidate(s, all_sims=True)
    got = Consolidator(s).consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert _first_diff(want, got) is None, _first_diff(want, got)
