"""Oracle Validation.IsValid + ValidateCommand (validation.go:68-180) vs the TTL-wait tests of
consolidation_test.go:2212-2562 (transcribed in tests/golden/make_consolidation_fixtures.py): the
command the oracle computes on `before` must be the Go test's, and re-checking it against `after`
must reach the Go test's verdict."""
import json
import os
import sys

import pytest

from oracle import bridge

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_consolidation_fixtures as mcf  # noqa: E402

FIXTURES = json.load(open(os.path.join(HERE, "golden", "validation_scenarios.json")))
SCENARIOS = {s["name"]: s for s in mcf.validation_scenarios()}


def final_command(doc):
    """Disruption controller method order: multi-node consolidation, then single-node."""
    m = doc["multi"]["command"]
    return m if m["action"] != "no-op" else doc["single"]["command"]


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_reference_validation_scenarios(fx):
    scn = SCENARIOS[fx["name"]]
    assert scn["expect"] == fx["expect"]
    doc, _ = bridge.consolidate(scn["before"])
    cmd = final_command(doc)
    assert cmd["action"] == fx["expect"]["command"], json.dumps(doc)[:2000]
    got = bridge.validate(scn["after"], cmd)
    assert got["valid"] == fx["expect"]["valid"], got
    assert got["reason"] == fx["expect"]["reason"], got


def test_subset_rule_and_no_replacement_expected():
    """A replace command whose options are not all offered by the re-simulated NodeClaim is refused
    (instanceTypesAreSubset validation.go:183-187); a delete command meeting a NodeClaim too."""
    scn = SCENARIOS["unchanged-can-replace-node"]
    doc, _ = bridge.consolidate(scn["before"])
    cmd = final_command(doc)
    assert bridge.validate(scn["after"], cmd)["valid"]
    bad = json.loads(json.dumps(cmd))
    bad["replacement"]["instanceTypeOptions"].append("no-such-type")
    assert bridge.validate(scn["after"], bad)["reason"] == "instance-types-not-subset"
    nodel = {"action": "delete", "candidates": cmd["candidates"]}
    assert bridge.validate(scn["after"], nodel)["reason"] == "replacement-needed"
    assert bridge.validate(scn["after"], {"candidates": []})["reason"] == "no-candidates"
