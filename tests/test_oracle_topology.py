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
