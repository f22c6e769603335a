"""GPU parity for the pod objects multi-node consolidation's probes share.

The reference's firstNConsolidationOption (multinodeconsolidation.go:101-135) hands every probe the same
Candidate.pods objects (types.go:114-126, helpers.go:102-104) and Preferences.Relax mutates them in place
(preferences.go:60-147): a pod one probe relaxed starts the next probe relaxed.  ks_cons.cpp carry_walk resolves
the search over the pass's records and re-runs on the GPU each probe that holds such a pod, from the carried
relaxation states (KsWork::sstart); every simulation's NewTopology starts with the groups its pods' starting
states create (KsWork::tact).  GPU == oracle (oracle/consolidation.inc CarriedPods) on the path, the commands and
every simulation."""
import json

import pytest

import carry_scenarios as cs
from karpenter_amd import Consolidator
from oracle import bridge

pytestmark = pytest.mark.gpu


def _diff(a, b, path=""):
    if type(a) != type(b):
        return "%s: %r vs %r" % (path, a, b)
    if isinstance(a, dict):
        for k in sorted(set(a) | set(b)):
            if a.get(k) != b.get(k):
                return _diff(a.get(k), b.get(k), path + "." + k)
    elif isinstance(a, list):
        if len(a) != len(b):
            return "%s: len %d vs %d" % (path, len(a), len(b))
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                return _diff(x, y, "%s[%d]" % (path, i))
    return "%s: %r vs %r" % (path, a, b)


def _check(snap, all_sims=True):
    s = json.dumps(snap)
    want, _ = bridge.consolidate(s, all_sims=all_sims)
    c = Consolidator(s)
    got = c.consolidate(all_sims=all_sims)
    got.pop("kernel_ms")
    assert got == want, _diff(want, got)
    carried = sum(1 for p in want["multi"]["path"] if p["carried"])
    assert c.last_reruns >= carried, (c.last_reruns, carried)
    return want, c


@pytest.mark.parametrize("volumes", [False, True])
@pytest.mark.parametrize("variant", [0, 1])
@pytest.mark.parametrize("kind", cs.KINDS)
def test_constructed_carry_scenarios(kind, variant, volumes):
    want, c = _check(cs.make(kind, variant, volumes=volumes))
    assert want["multi"]["path"][1]["carried"]
    assert c.last_reruns >= 1
    # without all_sims the multi-node "sims" are the probes the reference runs (the carried one included)
    _check(cs.make(kind, variant, volumes=volumes), all_sims=False)


@pytest.mark.parametrize("variant", [0, 1])
def test_group_created_late_in_one_simulation(variant):
    """cand-b's single-node simulation creates pod A's spread group only at B's relaxation (A stays bound
    elsewhere): a late group there with no node hostnames registered, although the problem's build created it
    up front (KsWork::tact + the hostname entries of sim_topology)."""
    want, _ = _check(cs.late_group_cluster(variant))
    assert want["single"]["sims"][1]["action"] == "replace"


@pytest.mark.parametrize("topology", [True, False])
@pytest.mark.parametrize("seed", range(16))
def test_random_carry_clusters(seed, topology):
    _check(cs.random_cluster(seed, topology=topology))


def test_random_carry_clusters_change_outcomes():
    """The random family above does reach probes whose carried outcome differs from the pristine one."""
    diffs = 0
    for seed in range(16):
        for topology in (True, False):
            doc, _ = bridge.consolidate(json.dumps(cs.random_cluster(seed, topology=topology)), all_sims=True)
            pristine = {len(x["candidates"]) - 1: x for x in doc["multi"]["sims"]}
            for p in doc["multi"]["path"]:
                q = {k: v for k, v in p.items() if k not in ("mid", "carried")}
                diffs += p["carried"] and q != pristine[p["mid"]]
    assert diffs >= 3


@pytest.mark.parametrize("seed", [1, 4, 23, 38])
def test_sharded_records_carry(seed):
    """World 2 on one GPU: two handles run the two shards, rank 0 decides over the gathered records.  A probe
    that relaxed pods and ran on the other rank is re-run here for its final states; the decision equals the
    world-1 one."""
    s = json.dumps(cs.random_cluster(seed, topology=seed % 2 == 0))
    want, _ = bridge.consolidate(s, all_sims=False)
    a, b = Consolidator(s), Consolidator(s)
    ra, _ = a.run(0, 2)
    ra = bytes(ra)
    rb, _ = b.run(1, 2)
    recs = ra + bytes(rb)
    owner = {0: a, 1: b}
    got = a.decide(recs, 2, fetch=lambda sim: owner[sim % 2].claim_requirements(sim))
    assert got["multi"] == want["multi"], _diff(want["multi"], got["multi"])
    assert got["single"]["command"] == want["single"]["command"]
