"""Multi-node consolidation's probes share the candidates' pod objects (oracle side).

The reference's binary search (multinodeconsolidation.go:101-135) appends the same *v1.Pod pointers, listed once
per pass by NewCandidate (types.go:114-126), to every probe's simulation (helpers.go:102-104); Preferences.Relax
mutates them in place (preferences.go:60-147).  oracle/consolidation.inc carries the pod objects from probe to
probe (CarriedPods).  tests/carry_scenarios.py builds clusters where that changes the chosen command."""
import json

import pytest

import carry_scenarios as cs
from oracle import bridge


def _pristine(doc, mid):
    for x in doc["multi"]["sims"]:
        if len(x["candidates"]) == mid + 1:
            return x
    raise KeyError(mid)


@pytest.mark.parametrize("kind", cs.KINDS)
def test_carried_probe_changes_the_command(kind):
    """Probe 1 (candidates 0-2) relaxes P; probe 2 (candidates 0-1) starts from the relaxed P.  Variant 0: the
    carried probe deletes both candidates where the pristine pods would need a replacement (spread-any: the
    reverse capacity layout, variant 1; late-carry: both, the pristine P's relaxed group is created mid-Solve
    without the keep nodes' hostnames); the other variant is the control where both agree."""
    diff_variants = {"spread-any": (1,), "late-carry": (0, 1)}.get(kind, (0,))
    for variant in (0, 1):
        doc, _ = bridge.consolidate(json.dumps(cs.make(kind, variant)), all_sims=True)
        path = doc["multi"]["path"]
        assert [p["mid"] for p in path] == [2, 1]
        assert not path[0]["carried"] and path[1]["carried"]
        second = {k: v for k, v in path[1].items() if k not in ("mid", "carried")}
        if variant in diff_variants:
            assert second["action"] == "delete"
            assert _pristine(doc, 1)["action"] == "replace"
            assert second != _pristine(doc, 1)
            assert doc["multi"]["command"] == {"action": "delete", "candidates": ["cand-0", "cand-1"]}
        else:
            assert second == _pristine(doc, 1)


@pytest.mark.parametrize("kind", cs.KINDS)
def test_sequential_path_equals_threaded_checker(kind):
    """The threaded checker (used for the full-size digests) carries only relaxed pods and reuses the pristine
    prefix simulations; the sequential mode carries every pod object exactly as the Solve left it (the in-place
    preferred-term sort and the re-injected volume requirements included).  Same path, same commands."""
    for variant in (0, 1):
        s = json.dumps(cs.make(kind, variant))
        seq, _ = bridge.consolidate(s, all_sims=True, threads=1)
        thr, _ = bridge.consolidate(s, all_sims=True, threads=3)
        assert seq["multi"] == thr["multi"]
        assert seq["single"]["command"] == thr["single"]["command"]


def test_non_all_sims_reports_the_path():
    """Without all_sims the multi-node "sims" are the probes the reference ran, carried ones included."""
    doc, _ = bridge.consolidate(json.dumps(cs.make("pref-node", 0)), all_sims=False)
    path = [{k: v for k, v in p.items() if k not in ("mid", "carried")} for p in doc["multi"]["path"]]
    assert doc["multi"]["sims"] == path


def test_volume_pods_carry_exactly():
    """A relaxed candidate pod with a bound PVC: VolumeTopology.Inject appends its zone requirement to the
    required terms again in every probe (volumetopology.go:68-71).  The exact sequential carry (the re-injected
    object) and the threaded checker's (a relaxed pod's object, pristine otherwise) agree."""
    for kind in ("pref-node", "pref-node-2"):
        snap = cs.make(kind, 0, volumes=True)
        s = json.dumps(snap)
        seq, _ = bridge.consolidate(s, all_sims=True, threads=1)
        thr, _ = bridge.consolidate(s, all_sims=True, threads=3)
        assert seq["multi"] == thr["multi"]
        assert seq["multi"]["path"][1]["carried"]
