"""GPU parity for consolidation: the batched simulations + on-GPU computeConsolidation decisions,
replayed by the host selection, must equal the oracle's restatement of pkg/controllers/disruption
(oracle/consolidation.inc) exactly: candidate order and disruption costs, every simulation outcome
(allNonPendingScheduled, #NewNodeClaims, NewNodeClaims[0] options and requirements) and the chosen
multi-node and single-node commands (action, candidates, replacement options and requirements)."""
import json
import os
import sys

import pytest

from karpenter_amd import Consolidator, synth
from oracle import bridge

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_consolidation_fixtures as mcf  # noqa: E402

FIXTURES = json.load(open(os.path.join(HERE, "golden", "consolidation_scenarios.json")))
SCENARIOS = {s["name"]: s for s in mcf.scenarios()}


def _both(snap, all_sims):
    s = json.dumps(snap)
    want, _ = bridge.consolidate(s, all_sims=all_sims)
    got = Consolidator(s).consolidate(all_sims=all_sims)
    got.pop("kernel_ms")
    return want, got


def _explain(a, b, path=""):
    """Pinpoint the first difference between two JSON values."""
    if type(a) != type(b):
        return "%s: %r vs %r" % (path, a, b)
    if isinstance(a, dict):
        for k in sorted(set(a) | set(b)):
            if a.get(k) != b.get(k):
                return _explain(a.get(k), b.get(k), path + "." + k)
    elif isinstance(a, list):
        if len(a) != len(b):
            sa, sb = set(map(json.dumps, a)), set(map(json.dumps, b))
            return "%s: len %d vs %d; only want %s; only got %s" % (path, len(a), len(b), sorted(sa - sb)[:5],
                                                                   sorted(sb - sa)[:5])
        for i, (x, y) in enumerate(zip(a, b)):
            if x != y:
                return _explain(x, y, "%s[%d]" % (path, i))
    return "%s: %r vs %r" % (path, a, b)


def _first_diff(want, got):
    if want == got:
        return None
    return _explain(want, got)


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_reference_consolidation_scenarios_gpu(fx):
    """consolidation_test.go known answers (tests/golden), GPU path vs oracle and vs the expectation."""
    scn = SCENARIOS[fx["name"]]
    for all_sims in (False, True):
        want, got = _both(scn["snapshot"], all_sims)
        d = _first_diff(want, got)
        assert d is None, d
    m = got["multi"]["command"]
    cmd = m if m["action"] != "no-op" else got["single"]["command"]
    assert cmd["action"] == fx["expect"]["action"]
    assert sorted(cmd["candidates"]) == sorted(fx["expect"]["candidates"])


CASES = [
    dict(n_nodes=12, pods_per_node=6, n_its=40, it_range=(8, 24), seed=1),
    dict(n_nodes=24, pods_per_node=10, n_its=60, it_range=(6, 30), seed=2, spot_frac=0.6),
    dict(n_nodes=30, pods_per_node=12, n_its=80, it_range=(10, 40), seed=3, n_pending=5),
    dict(n_nodes=20, pods_per_node=8, n_its=50, it_range=(5, 20), seed=4, uninitialized_frac=0.2, not_ready_frac=0.2),
    dict(n_nodes=25, pods_per_node=10, n_its=60, it_range=(8, 30), seed=5, pod_selectors=True),
    dict(n_nodes=16, pods_per_node=15, n_its=40, it_range=(2, 10), seed=6, expire_after="48h"),
    dict(n_nodes=40, pods_per_node=5, n_its=100, it_range=(20, 60), seed=7, spot_frac=1.0),
    dict(n_nodes=18, pods_per_node=9, n_its=40, it_range=(4, 16), seed=8, limits={"cpu": "300"}),
]


@pytest.mark.parametrize("case", CASES, ids=["c%d" % c["seed"] for c in CASES])
def test_random_cluster_parity(case):
    snap = synth.cluster_snapshot(**case)
    for all_sims in (True, False):
        want, got = _both(snap, all_sims)
        d = _first_diff(want, got)
        assert d is None, d


TOPO_CASES = [
    dict(n_nodes=40, pods_per_node=5, n_its=60, seed=0, n_pending=3, topology=8),
    dict(n_nodes=40, pods_per_node=8, n_its=60, seed=1, n_pending=3, topology=16),
    dict(n_nodes=40, pods_per_node=10, n_its=60, seed=2, n_pending=3, topology=4),
    dict(n_nodes=40, pods_per_node=3, n_its=60, seed=3, n_pending=3, topology=12),
    dict(n_nodes=24, pods_per_node=10, n_its=60, it_range=(6, 30), seed=21, spot_frac=0.6, topology=6),
    dict(n_nodes=30, pods_per_node=12, n_its=80, it_range=(10, 40), seed=22, n_pending=5, topology=24),
    dict(n_nodes=20, pods_per_node=8, n_its=50, it_range=(5, 20), seed=23, uninitialized_frac=0.2,
         not_ready_frac=0.2, topology=10),
    dict(n_nodes=25, pods_per_node=10, n_its=60, it_range=(8, 30), seed=24, pod_selectors=True, topology=3),
    dict(n_nodes=16, pods_per_node=15, n_its=40, it_range=(2, 10), seed=25, topology=2),
    dict(n_nodes=60, pods_per_node=4, n_its=100, it_range=(20, 60), seed=26, topology=40),
]


@pytest.mark.parametrize("case", TOPO_CASES, ids=["t%d" % c["seed"] for c in TOPO_CASES])
def test_topology_cluster_parity(case):
    """Simulations whose pods carry spread / pod affinity / anti-affinity over a cluster whose bound pods
    seed NewTopology: every simulation's counts exclude its own pods (topology.go:72-75) and its removed
    nodes' hostnames are no longer registered."""
    snap = synth.cluster_snapshot(**case)
    for all_sims in (True, False):
        want, got = _both(snap, all_sims)
        d = _first_diff(want, got)
        assert d is None, d


def _volume_cluster(seed, n_nodes, ppn, topology=0):
    import numpy as np

    import problems
    snap = synth.cluster_snapshot(n_nodes, ppn, n_its=40, it_range=(4, 20), seed=seed, n_pending=2, topology=topology)
    pods = snap["pendingPods"] + [p for n in snap["stateNodes"] for p in n["pods"]]
    snap["volumeDrivers"] = problems.add_volumes(np.random.default_rng(seed), pods, snap["stateNodes"])
    return snap


@pytest.mark.parametrize("seed", [61, 62, 63])
def test_pdb_cluster_parity(seed):
    """PodDisruptionBudgets filter the candidates (filterCandidates helpers.go:47-71) before any simulation."""
    snap = synth.cluster_snapshot(30, 6, n_its=40, it_range=(4, 30), seed=seed, n_pending=2, pdbs=True)
    for all_sims in (True, False):
        want, got = _both(snap, all_sims)
        d = _first_diff(want, got)
        assert d is None, d


VOL_CASES = [(41, 12, 5, 0), (42, 16, 4, 0), (43, 10, 6, 0), (44, 14, 4, 6), (45, 8, 8, 0), (46, 12, 3, 4)]


@pytest.mark.parametrize("seed,n_nodes,ppn,topo", VOL_CASES, ids=["v%d" % c[0] for c in VOL_CASES])
def test_volume_cluster_parity(seed, n_nodes, ppn, topo):
    """Simulations whose pods mount PVCs of limited CSI drivers onto nodes with CSINode limits and an
    existing usage (volumeusage.go:183-227): each simulation's usage is copy-on-write over the shared one."""
    snap = _volume_cluster(seed, n_nodes, ppn, topo)
    for all_sims in (True, False):
        want, got = _both(snap, all_sims)
        d = _first_diff(want, got)
        assert d is None, d


def test_sharded_runs_gather_to_the_same_decision():
    """Ranks r of world W run simulations s % W == r; the [rank][slot] gather decides identically."""
    snap = json.dumps(synth.cluster_snapshot(30, 8, n_its=60, it_range=(6, 30), seed=11, spot_frac=0.5))
    c = Consolidator(snap)
    one = c.decide(c.run(0, 1)[0], 1, all_sims=True)
    for world in (2, 3, 8):
        ranks = [Consolidator(snap) for _ in range(world)]  # one handle per "GPU"
        recs = b"".join(ranks[r].run(r, world)[0] for r in range(world))
        got = c.decide(recs, world, all_sims=True, fetch=lambda s: ranks[s % world].claim_requirements(s))
        assert got == one


def test_c5_shape_at_scale_properties():
    """1000-node slice of the C5 cluster: every single-node simulation is evaluated.  The cluster has the
    headroom for any one node's 20 pods, so every single-node simulation reschedules all of them onto
    the remaining nodes without a new NodeClaim (a delete), and the multi-node search reaches the
    largest prefix (101 candidates, multinodeconsolidation.go:93-95) as a delete — as the oracle
    computes for this cluster (the full 5k-node pass is compared to it in test_full_size_gpu.py)."""
    snap = synth.cluster_snapshot(1000, 20, 400, seed=4205)
    c = Consolidator(json.dumps(snap))
    assert c.num_candidates == 1000 and c.num_sims == 1000 + 100
    doc = c.consolidate(all_sims=True)
    assert len(doc["single"]["sims"]) == 1000
    assert all(s["allNonPendingScheduled"] and s["newNodeClaims"] == 0 for s in doc["single"]["sims"])
    assert doc["single"]["command"]["action"] == "delete"
    assert doc["single"]["command"]["candidates"] == [doc["candidates"][0]["name"]]
    assert doc["multi"]["command"]["action"] == "delete" and len(doc["multi"]["command"]["candidates"]) == 101
    costs = [x["disruptionCost"] for x in doc["candidates"]]
    assert costs == sorted(costs)
    # determinism
    assert c.consolidate(all_sims=True)["single"] == doc["single"]


# ---- Validation.IsValid + ValidateCommand (validation.go:68-180) -----------------------------------
VFIXTURES = json.load(open(os.path.join(HERE, "golden", "validation_scenarios.json")))
VSCENARIOS = {s["name"]: s for s in mcf.validation_scenarios()}


def _final(doc):
    m = doc["multi"]["command"]
    return m if m["action"] != "no-op" else doc["single"]["command"]


@pytest.mark.parametrize("fx", VFIXTURES, ids=[f["name"] for f in VFIXTURES])
def test_reference_validation_scenarios_gpu(fx):
    """consolidation_test.go TTL-wait known answers: the GPU computes the command on `before` and
    re-simulates it on `after`; both steps equal the oracle and the Go test's verdict."""
    scn = VSCENARIOS[fx["name"]]
    want, got = _both(scn["before"], False)
    assert _first_diff(want["multi"], got["multi"]) is None
    assert _first_diff(want["single"], got["single"]) is None
    cmd = _final(got)
    assert cmd["action"] == fx["expect"]["command"]
    v_want = bridge.validate(scn["after"], cmd)
    v_got = Consolidator(json.dumps(scn["after"])).validate(cmd)
    assert _first_diff(v_want, v_got) is None, _first_diff(v_want, v_got)
    assert (v_got["valid"], v_got["reason"]) == (fx["expect"]["valid"], fx["expect"]["reason"])


def _perturb(snap, variant, seed):
    import copy
    import random
    after = copy.deepcopy(snap)
    rng = random.Random(seed)
    if variant == "pending":  # new pending pods arrive during the wait
        after["pendingPods"] = list(after.get("pendingPods", [])) + [
            synth.pod(900000 + i, cpu=rng.choice(["1", "2", "4"]), mem="1Gi") for i in range(3)]
    elif variant == "full":  # a third of the nodes fill up
        for n in after["stateNodes"]:
            if rng.random() < 0.34:
                n["available"]["pods"] = "0"
    elif variant == "nominated":
        for n in after["stateNodes"]:
            n["nominated"] = rng.random() < 0.2
    return after


@pytest.mark.parametrize("seed,variant", [(s, v) for s in (61, 62, 63) for v in ("same", "pending", "full", "nominated")])
def test_random_validation_parity(seed, variant):
    """Commands from a random cluster (multi-node, single-node and every single-node simulation's
    replacement) re-checked on a perturbed cluster: GPU ValidateCommand == oracle, field by field."""
    snap = synth.cluster_snapshot(24, 6, n_its=40, it_range=(4, 30), seed=seed, spot_frac=0.3, n_pending=1)
    doc = Consolidator(json.dumps(snap)).consolidate(all_sims=True)
    cmds = [doc["multi"]["command"], doc["single"]["command"]]
    for sim in doc["single"]["sims"][:8]:
        c = {"action": "replace", "candidates": sim["candidates"]}
        if sim.get("claim0"):
            c["replacement"] = {"instanceTypeOptions": sim["claim0"]["instanceTypeOptions"][:5]}
        cmds.append(c)
    after = _perturb(snap, variant, seed)
    h = Consolidator(json.dumps(after))
    reasons = set()
    for cmd in cmds:
        v_want = bridge.validate(after, cmd)
        v_got = h.validate(cmd)
        assert _first_diff(v_want, v_got) is None, (cmd, _first_diff(v_want, v_got))
        reasons.add(v_got["reason"])
    # the handle's own pass is untouched by the validation runs
    again = h.consolidate(all_sims=False)
    want, _ = bridge.consolidate(json.dumps(after), all_sims=False)
    assert again["single"]["command"] == want["single"]["command"]
    assert reasons


@pytest.mark.parametrize("seed", (3, 4))
def test_consolidation_over_derived_cluster_state(seed):
    """Consolidation over stateNodes derived by ks_cluster_state from Node / NodeClaim / Pod listings
    (cluster-state accounting, pkg/controllers/state): GPU decisions == oracle."""
    import test_cluster_state as tcs
    its = mcf.assorted()[:64]
    base = mcf.snapshot(its, [])
    c = tcs.consolidatable(tcs.random_cluster(seed, n=16), its, seed)
    from karpenter_amd import cluster_state
    state = cluster_state(json.dumps(c))
    base["stateNodes"] = state
    base["candidates"] = [n["name"] for n in state]
    want, got = _both(base, True)
    assert _first_diff(want, got) is None, _first_diff(want, got)


def test_consolidation_from_raw_listings():
    """End to end from Node / NodeClaim / Pod listings: ks_cons_create derives the StateNodes itself;
    the decisions equal the oracle's over its own derived state."""
    import test_cluster_state as tcs
    with_state, with_cluster = tcs._cons_inputs(7)
    want, _ = bridge.consolidate(json.dumps(with_state), all_sims=True)
    got = Consolidator(json.dumps(with_cluster)).consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert _first_diff(want, got) is None, _first_diff(want, got)


def test_validation_at_scale_unchanged_cluster():
    """A command validated against the cluster it was computed on is valid (validation.go:120-180 on an
    unchanged cluster), for both the multi-node and the single-node command, and the GPU verdict equals
    the oracle's at 600 nodes x 20 pods (the C5 shape, scaled down for the oracle)."""
    snap = json.dumps(synth.config5(600))
    h = Consolidator(snap)
    doc = h.consolidate()
    for kind in ("multi", "single"):
        cmd = doc[kind]["command"]
        if cmd["action"] == "no-op":
            continue
        got = h.validate(cmd)
        assert got["valid"], (kind, got)
        assert _first_diff(bridge.validate(snap, cmd), got) is None


@pytest.mark.parametrize("seed,topo", [(71, 0), (72, 8), (73, 24)])
def test_validation_of_arbitrary_candidate_subsets(seed, topo):
    """Commands whose candidates are not a prefix of the disruption-cost order (a command from an earlier
    snapshot, whose order has since changed): the re-simulation removes an arbitrary subset, with its
    topology counts and hostnames, and its verdict equals the oracle's."""
    import random
    snap = synth.cluster_snapshot(20, 6, n_its=40, it_range=(4, 30), seed=seed, n_pending=1, topology=topo)
    s = json.dumps(snap)
    h = Consolidator(s)
    names = [c["name"] for c in bridge.consolidate(s)[0]["candidates"]]
    rng = random.Random(seed)
    for _ in range(10):
        cands = rng.sample(names, rng.randint(1, min(5, len(names))))
        cmd = {"action": "delete", "candidates": cands}
        want, got = bridge.validate(s, cmd), h.validate(cmd)
        assert _first_diff(want, got) is None, (cands, _first_diff(want, got))


def test_validate_keeps_the_pass_launch():
    """ks_cons_validate re-simulates in a launch of its own: after run -> validate on one handle, the
    pass's records still decide identically, and the requirement records and counters the decision
    reads (ks_cons_claim_requirements, ks_cons_sim_counters) still come from the pass's launch."""
    snap = json.dumps(synth.cluster_snapshot(24, 10, n_its=60, it_range=(6, 30), seed=2, spot_frac=0.6))
    c = Consolidator(snap)
    recs, _ = c.run(0, 1)
    before = c.decide(recs, 1, all_sims=True)
    need = c.needed_sims(recs, 1, all_sims=True)
    assert need, "the scenario's multi-node command is a replace, which needs a requirement record"
    reqs = {s: c.claim_requirements(s) for s in need}
    counters = c.sim_counters(need[0])
    for cmd in (before["multi"]["command"], before["single"]["command"]):
        v = c.validate(cmd)
        assert v["valid"], v
    assert c.decide(recs, 1, all_sims=True) == before
    assert {s: c.claim_requirements(s) for s in need} == reqs
    assert c.sim_counters(need[0]) == counters
    want, _ = bridge.consolidate(snap, all_sims=True)
    got = dict(before)
    assert _first_diff(want, got) is None


@pytest.mark.parametrize("clock", [(60.0, 180.0, 0.0), (60.0, 180.0, 25.0), (60.0, 180.0, 100.0), (60.0, 180.0, 250.0),
                                   (1.0, 2.0, 0.5)])
@pytest.mark.parametrize("which", [("c", 1), ("c", 6), ("t", 1), ("t", 24)])
def test_consolidation_timeouts_parity(clock, which):
    """MultiNodeConsolidation's 1 min and SingleNodeConsolidation's 3 min timeouts (multinodeconsolidation.go:
    99-110: return the last saved command; singlenodeconsolidation.go:58-65: abandon) on a virtual clock
    that advances per simulation the sequential replay consults: GPU replay == oracle."""
    case = [c for c in (CASES if which[0] == "c" else TOPO_CASES) if c["seed"] == which[1]][0]
    snap = json.dumps(synth.cluster_snapshot(**case))
    want = bridge.consolidate_clock(snap, *clock)
    got = Consolidator(snap).consolidate(clock=clock)
    got.pop("kernel_ms")
    assert _first_diff(want, got) is None, _first_diff(want, got)


def test_records_kept_in_handle_gpu():
    """ks_cons_run with records NULL (world 1): decide / alg_bytes read the handle's pinned records; same
    decision and bytes as with the records copied out."""
    snap = synth.cluster_snapshot(30, 6, n_its=40, seed=77, n_pending=2)
    c = Consolidator(json.dumps(snap))
    recs, _ = c.run(0, 1)
    want = c.decide(bytes(recs), 1, all_sims=True)
    wb = c.alg_bytes(bytes(recs))
    none, _ = c.run(0, 1, keep=True)
    assert none is None
    assert c.decide(None, 1, all_sims=True) == want
    assert c.alg_bytes(None) == wb


def test_decide_without_sims_gpu():
    """KS_CONS_NO_SIMS: the per-simulation lists are left out, the commands are those of the full output."""
    snap = synth.cluster_snapshot(30, 6, n_its=40, seed=78, n_pending=2, spot_frac=0.4)
    c = Consolidator(json.dumps(snap))
    recs, _ = c.run(0, 1)
    full = c.decide(recs, 1)
    lean = c.decide(recs, 1, sims=False)
    for m in ("multi", "single"):
        assert lean[m]["command"] == full[m]["command"]
        assert lean[m]["sims"] == []
