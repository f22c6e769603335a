"""Oracle consolidation vs the reference's consolidation_test.go assertions (transcribed in
tests/golden/make_consolidation_fixtures.py), plus internal consistency of the all-sims mode."""
import json
import os
import sys

import pytest

from oracle import bridge

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_consolidation_fixtures as mcf  # noqa: E402

FIXTURES = json.load(open(os.path.join(HERE, "golden", "consolidation_scenarios.json")))
SCENARIOS = {s["name"]: s for s in mcf.scenarios()}


def final_command(doc):
    """Disruption controller method order: multi-node consolidation, then single-node."""
    m = doc["multi"]["command"]
    return m if m["action"] != "no-op" else doc["single"]["command"]


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_reference_consolidation_scenarios(fx):
    scn = SCENARIOS[fx["name"]]
    assert scn["expect"] == fx["expect"]
    doc, _ = bridge.consolidate(scn["snapshot"])
    cmd = final_command(doc)
    exp = fx["expect"]
    assert cmd["action"] == exp["action"], json.dumps(doc)[:2000]
    assert sorted(cmd["candidates"]) == sorted(exp["candidates"])
    if "replacement_excludes" in exp:
        assert exp["replacement_excludes"] not in cmd["replacement"]["instanceTypeOptions"]
        assert cmd["replacement"]["instanceTypeOptions"]


def test_all_sims_mode_same_commands():
    """Simulating every candidate / prefix up front must not change the chosen commands."""
    from karpenter_amd import synth
    snap = synth.cluster_snapshot(24, 12, n_its=40, it_range=(8, 24), seed=7)
    a, _ = bridge.consolidate(snap, all_sims=False)
    b, _ = bridge.consolidate(snap, all_sims=True)
    assert a["multi"]["command"] == b["multi"]["command"]
    assert a["single"]["command"] == b["single"]["command"]
    assert len(b["single"]["sims"]) == 24
