"""The oracle reproduces the reference's own scheduling known answers (suite_test.go Binpacking and
Provider Specific Labels), with the fake provider's cheapest-option launch rule."""
import json
import os

import pytest

import scenario_check
from oracle import bridge

with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scenarios.json")) as f:
    SCENARIOS = json.load(f)


@pytest.mark.parametrize("scn", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_oracle_scenario(scn):
    res, _ = bridge.solve(scn["snapshot"])
    bad = scenario_check.check(scn, res)
    assert not bad, bad
