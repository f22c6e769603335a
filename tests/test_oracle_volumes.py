"""Oracle VolumeUsage restatement (volumeusage.go:82-227, existingnode.go:70-78,122) vs the reference's
suite_test.go VolumeUsage assertions (transcribed in tests/golden/make_volume_fixtures.py)."""
import json
import os
import sys

import pytest

from oracle import bridge

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_volume_fixtures as mvf  # noqa: E402

FIXTURES = json.load(open(os.path.join(HERE, "golden", "volume_scenarios.json")))
SCENARIOS = {s["name"]: s for s in mvf.scenarios()}


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_reference_volume_scenarios(fx):
    scn = SCENARIOS[fx["name"]]
    assert scn["expect"] == fx["expect"]
    res, _ = bridge.solve(scn["snapshot"])
    bad = mvf.check(scn, res)
    assert not bad, bad


def test_limits_are_what_splits_the_pods():
    """Without the CSINode limit the same pods all fit the existing node: the scenario pins the check."""
    scn = json.loads(json.dumps(SCENARIOS["volume-limits-multiple-nodes"]))
    scn["snapshot"]["stateNodes"][0]["volumeLimits"] = {}
    res, _ = bridge.solve(scn["snapshot"])
    assert len(res["newNodeClaims"]) == 0 and len(res["existingNodes"][0]["pods"]) == 6
