"""Oracle Topology restatement vs the reference's topology_test.go assertions (transcribed in
tests/golden/make_topology_fixtures.py): zonal / hostname / capacity-type spread incl. minDomains and
nil selectors, node-selector-limited spread, required / preferred / inverse pod anti-affinity."""
import json
import os
import sys

import pytest

from oracle import bridge

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_topology_fixtures as mtf  # noqa: E402

FIXTURES = json.load(open(os.path.join(HERE, "golden", "topology_scenarios.json")))
SCENARIOS = {s["name"]: s for s in mtf.scenarios()}


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_reference_topology_scenarios(fx):
    scn = SCENARIOS[fx["name"]]
    assert scn["expect"] == fx["expect"]
    res, _ = bridge.solve(scn["snapshot"])
    bad = mtf.check(scn, res)
    assert not bad, bad


@pytest.mark.parametrize("mode,seed", [(1, 0), (2, 11), (2, 12), (2, 13)])
def test_reference_assertions_hold_under_any_map_order(mode, seed):
    """the Go tests assert multisets, so their assertions must hold whichever minimal
    domain Go's random map iteration picks.  Re-running every transcribed scenario with other tie-breaks
    (largest name, seeded random) keeps them green, so the canonical choice the GPU reproduces is one
    member of the reference's feasible tie set, not an artefact the fixtures depend on."""
    try:
        bridge.set_tie_mode(mode, seed)
        failures = {}
        for fx in FIXTURES:
            scn = SCENARIOS[fx["name"]]
            res, _ = bridge.solve(scn["snapshot"])
            bad = mtf.check(scn, res)
            if bad:
                failures[fx["name"]] = bad
        assert not failures, failures
    finally:
        bridge.set_tie_mode(0)


def test_tie_modes_change_some_choice():
    """The alternative tie-breaks are live: on a zonal spread with several empty zones they place pods
    differently from the canonical order."""
    scn = next(s for s in SCENARIOS.values() if "zonal" in s["name"] or "zone" in s["name"])
    base, _ = bridge.solve(scn["snapshot"])
    try:
        bridge.set_tie_mode(1)
        alt, _ = bridge.solve(scn["snapshot"])
    finally:
        bridge.set_tie_mode(0)
    assert [c["requirementsString"] for c in base["newNodeClaims"]] != \
        [c["requirementsString"] for c in alt["newNodeClaims"]]
