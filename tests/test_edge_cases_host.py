"""Empty and ragged inputs on the host side (no device): the encoder accepts them and the oracle's
results are what the reference's code produces for them."""
import json

import pytest

import edge_cases
from karpenter_amd import inspect, inspect_consolidation
from oracle import bridge

SOLVE = edge_cases.solve_cases()
CONS = edge_cases.cons_cases()


@pytest.mark.parametrize("name", sorted(SOLVE))
def test_solve_edge_inputs_encode(name):
    snap = SOLVE[name]
    dims = inspect(json.dumps(snap))
    assert dims
    res, _ = bridge.solve(json.dumps(snap))
    placed = sum(len(c["pods"]) for c in res["newNodeClaims"])
    if name == "no-templates-no-nodes":
        # reference quirk: with no existing node and no template, add() falls through its loops and
        # returns the nil multierr (scheduler.go:285), so Solve records no error for a pod placed nowhere
        assert placed == 0 and not res["podErrors"]
        return
    # every pod is placed exactly once or has an error (scheduler.go:140-189)
    assert placed + len(res["podErrors"]) == len(snap["pods"])
    if name == "no-instance-types":
        assert placed == 0 and len(res["podErrors"]) == len(snap["pods"])
    if name == "one-unschedulable":
        assert "0" in res["podErrors"] or 0 in res["podErrors"]


@pytest.mark.parametrize("name", sorted(CONS))
def test_consolidation_edge_inputs(name):
    snap = json.dumps(CONS[name])
    got = inspect_consolidation(snap)
    want, _ = bridge.consolidate(snap, all_sims=True)
    assert [c["name"] for c in got["candidates"]] == [c["name"] for c in want["candidates"]]
    if name == "no-candidates":
        assert got["sims"] == 0
        assert want["multi"]["command"]["action"] == "no-op" and want["single"]["command"]["action"] == "no-op"
    if name == "one-candidate":
        assert got["multiPrefixes"] == 0 and got["sims"] <= 1
