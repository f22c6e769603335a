"""CPU tests of the consolidation host logic: candidate construction and the disruption-cost order
(NewCandidate types.go:54-113, disruptionCost helpers.go:137-177, sort.Slice consolidation.go:79-81)
must equal the oracle's, and the simulation plan must cover firstNConsolidationOption's search
space (multinodeconsolidation.go:87-137) plus one simulation per candidate."""
import json
import os
import sys

import pytest

from karpenter_amd import inspect_consolidation, synth
from oracle import bridge

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_consolidation_fixtures as mcf  # noqa: E402

SNAPS = [("scn-" + s["name"], s["snapshot"]) for s in mcf.scenarios()] + [
    ("rand-%d" % seed, synth.cluster_snapshot(n, 6, n_its=40, it_range=(4, 30), seed=seed, spot_frac=0.4,
                                               uninitialized_frac=0.1, n_pending=3, expire_after=exp))
    for seed, n, exp in [(21, 10, "720h"), (22, 40, "24h"), (23, 130, "2h30m")]] + [
    ("topo-%d" % seed, synth.cluster_snapshot(30, 6, n_its=40, it_range=(4, 30), seed=seed, n_pending=3, topology=apps))
    for seed, apps in [(31, 8), (32, 24)]] + [
    ("pdb-%d" % seed, synth.cluster_snapshot(40, 6, n_its=40, it_range=(4, 30), seed=seed, n_pending=2, pdbs=True))
    for seed in (51, 52, 53)]


def test_pdbs_block_candidates():
    """PDBLimits.CanEvictPods (pdblimits.go:58-84) inside filterCandidates (helpers.go:47-71): a budget with
    no disruptions left removes every node running a selected pod, unless the budget always allows
    evicting unhealthy pods and the pod is not Ready."""
    snap = synth.cluster_snapshot(40, 6, n_its=40, it_range=(4, 30), seed=51, pdbs=True)
    base = dict(snap)
    base.pop("podDisruptionBudgets")
    with_pdb = inspect_consolidation(json.dumps(snap))["candidates"]
    without = inspect_consolidation(json.dumps(base))["candidates"]
    assert 0 < len(with_pdb) < len(without)


@pytest.mark.parametrize("name,snap", SNAPS, ids=[n for n, _ in SNAPS])
def test_candidates_match_oracle(name, snap):
    s = json.dumps(snap)
    got = inspect_consolidation(s)
    want, _ = bridge.consolidate(s, all_sims=False)
    assert [(c["name"], c["disruptionCost"]) for c in got["candidates"]] == \
        [(c["name"], c["disruptionCost"]) for c in want["candidates"]]
    n = len(got["candidates"])
    hi = 0 if n < 2 else (min(n, 100) if n > 100 else n - 1)
    assert got["multiPrefixes"] == hi
    assert got["sims"] == n + hi


def test_prefix_cap_is_101_candidates():
    got = inspect_consolidation(json.dumps(synth.cluster_snapshot(150, 2, n_its=30, it_range=(4, 20), seed=5)))
    assert got["multiPrefixes"] == 100 and got["sims"] == 250


@pytest.mark.parametrize("name,snap", SNAPS, ids=[n for n, _ in SNAPS])
def test_pending_pods_encoded(name, snap):
    """Every simulation schedules the pending pods (SimulateScheduling, helpers.go:79-85): the encode must
    hold each of them, in snapshot order, with its own requests (RequestsForPods incl. pods=1)."""
    got = inspect_consolidation(json.dumps(snap))
    pend = snap.get("pendingPods", [])
    assert [p["name"] for p in got["pendingPods"]] == [p["metadata"]["name"] for p in pend]
    res = got["resources"]
    for p, q in zip(pend, got["pendingPods"]):
        asked = {}
        for c in p["spec"].get("containers", []):
            for k, v in c.get("resources", {}).get("requests", {}).items():
                asked[k] = asked.get(k, 0) + (0 if str(v).strip("0.m") == "" else 1)
        enc = dict(zip(res, q["requests"]))
        assert enc.get("pods") == 1
        for k, nz in asked.items():
            if nz and k in enc:
                assert enc[k] > 0, (name, p["metadata"]["name"], k)
