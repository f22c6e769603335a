"""GPU parity: the HIP Solve path through the C-ABI vs the oracle, bit-exact on the canonical
Results (NewNodeClaims in final order with pods / instance-type options / requests / requirements,
ExistingNodes with pods, PodErrors text).  Go map-order choices are canonicalised identically on
both sides."""
import json

import pytest

import problems
from karpenter_amd import Scheduler, synth
from oracle import bridge

pytestmark = pytest.mark.gpu


def _solve_both(snap):
    s = json.dumps(snap)
    want, _ = bridge.solve(s)
    got = Scheduler(s).solve()
    return problems.canonical(want), got


def _diff(want, got):
    g = got.canonical()
    if want == g:
        return None
    for key in ("newNodeClaims", "existingNodes", "podErrors"):
        if want[key] != g[key]:
            if isinstance(want[key], list):
                for i, (a, b) in enumerate(zip(want[key], g[key])):
                    if a != b:
                        return "%s[%d]: want %s\n got %s" % (key, i, json.dumps(a)[:1500], json.dumps(b)[:1500])
                return "%s: length %d vs %d" % (key, len(want[key]), len(g[key]))
            ks = sorted(set(want[key]) | set(g[key]), key=lambda x: int(x))
            for k in ks:
                if want[key].get(k) != g[key].get(k):
                    return "%s[%s]: want %r\n got %r" % (key, k, want[key].get(k), g[key].get(k))
    return "differs"


@pytest.mark.parametrize("seed", list(range(48)))
def test_random_problem_parity(seed):
    want, got = _solve_both(problems.random_problem(seed))
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", list(range(200, 216)))
def test_host_ports_parity(seed):
    """HostPortUsage on existing nodes and in-flight NodeClaims (hostportusage.go:74-85)."""
    want, got = _solve_both(problems.random_problem(seed, n_pods=150, n_nodes=int(seed % 3) * 6, host_ports=True))
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", [100, 101, 102, 103])
def test_random_problem_parity_larger(seed):
    want, got = _solve_both(problems.random_problem(seed, n_pods=800, n_its=120, n_nodes=30))
    d = _diff(want, got)
    assert d is None, d


def test_config3_selectors_affinity_taints():
    """C3 shape (BASELINE.json configs[2]) at 1500 pods: 800 instance types x 8 offerings, 3 tainted
    weighted NodePools, selectors / required + preferred affinity / tolerations."""
    want, got = _solve_both(synth.config3(1500))
    d = _diff(want, got)
    assert d is None, d


def test_config3_long_claim_sorts():
    """C3 at 4000 pods: ~200 NodeClaims, so the per-placement sort.Slice (scheduler.go:247) runs the
    wave-parallel partialInsertionSort on long arrays, and the wave-parallel exact pdqsort (partition,
    partitionEqual, reversal, recursion) when choosePivot's samples straddle a descent."""
    want, got = _solve_both(synth.config3(4000))
    d = _diff(want, got)
    assert d is None, d
    assert got.stats["sortsWithDescent"] > 100
    assert got.stats["sortsExact"] > 0


def test_config1_benchmark_scheduling_2000():
    """BenchmarkScheduling2000 (scheduling_benchmark_test.go:72-74,116-182)."""
    want, got = _solve_both(synth.config1())
    assert _diff(want, got) is None
    assert len(got.pod_errors) == 0


def test_config2_10k_parity():
    want, got = _solve_both(synth.config2(10000))
    assert _diff(want, got) is None


def test_config2_full_size_properties():
    """50k pods x 400 ITs: size-independent properties (oracle parity is checked at 10k)."""
    snap = synth.config2(50000)
    got = Scheduler(snap).solve()
    placed = [p for c in got.new_nodeclaims for p in c["pods"]]
    assert sorted(placed) == list(range(50000))  # every pod placed exactly once
    assert not got.pod_errors
    its = {it["name"]: it for it in snap["instanceTypes"]}
    for c in got.new_nodeclaims:
        # the claim's options all fit its accumulated requests (Fits, resources.go:162-175)
        cpu_m = int(c["requests"]["cpu"].rstrip("m")) if c["requests"]["cpu"].endswith("m") else int(c["requests"]["cpu"]) * 1000
        for name in c["instanceTypeOptions"]:
            cap_m = int(its[name]["capacity"]["cpu"]) * 1000 - 100
            assert cpu_m <= cap_m
    # determinism: a second solve is identical
    again = Scheduler(snap).solve()
    assert again.canonical() == got.canonical()


def test_replicas_identical():
    snap = problems.random_problem(7)
    sch = Scheduler(snap)
    one = sch.solve(replicas=1).canonical()
    many = sch.solve(replicas=64).canonical()
    assert one == many


with open(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "scenarios.json")) as _f:
    SCENARIOS = json.load(_f)


@pytest.mark.parametrize("scn", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_reference_scenarios_gpu(scn):
    """suite_test.go known answers through the HIP path, plus bit-exact vs the oracle."""
    import scenario_check

    want, got = _solve_both(scn["snapshot"])
    assert scenario_check.check(scn, got.canonical()) == []
    assert _diff(want, got) is None


# (seed, budget): claims exceed Plan::KL (checked below via ks_problem_inspect's plans)
@pytest.mark.parametrize("seed,budget", [(201, 6000), (203, 14000), (206, 6000), (242, 9000), (251, 9000),
                                         (251, 14000)])
def test_small_lds_budget_parity(seed, budget):
    """Small LDS budgets move claim state past Plan::KL to HBM and the instance-type tables out of
    LDS; decisions must not change."""
    snap = problems.random_problem(seed, n_pods=400, n_its=30, n_nodes=5)
    from karpenter_amd import inspect
    plan = inspect(snap)["plans"][str(budget)]
    s = json.dumps(snap)
    want, _ = bridge.solve(s)
    assert plan["KL"] < len(want["newNodeClaims"]) <= plan["KO"]
    got = Scheduler(s).solve(lds_budget=budget)
    d = _diff(problems.canonical(want), got)
    assert d is None, d


def test_small_lds_budget_config2_overflow():
    """C2 at 10k with ~6 KB of LDS: claims past KL=19 live in HBM, sorted Allocatable lists too."""
    s = json.dumps(synth.config2(10000))
    want, _ = bridge.solve(s)
    assert len(want["newNodeClaims"]) > 19
    got = Scheduler(s).solve(lds_budget=6000)
    assert _diff(problems.canonical(want), got) is None


@pytest.mark.parametrize("seed", list(range(300, 316)))
def test_volume_limits_parity(seed):
    """VolumeUsage on existing nodes (volumeusage.go:82-227, existingnode.go:70-78,122): shared and
    ephemeral claims, unresolved / driverless claims, nodes already over a limit."""
    want, got = _solve_both(problems.random_problem(seed, n_pods=150, n_nodes=12 + seed % 5, volumes=True))
    d = _diff(want, got)
    assert d is None, d


def _volume_scenarios():
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import make_volume_fixtures as mvf
    return mvf


@pytest.mark.parametrize("name", [s["name"] for s in _volume_scenarios().scenarios()])
def test_volume_reference_scenarios_gpu(name):
    """suite_test.go VolumeUsage scenarios on the GPU: the Go assertions and equality with the oracle."""
    mvf = _volume_scenarios()
    scn = {s["name"]: s for s in mvf.scenarios()}[name]
    want, got = _solve_both(scn["snapshot"])
    d = _diff(want, got)
    assert d is None, d
    assert not mvf.check(scn, want)


def test_config1_literal_benchmark_pods():
    """BenchmarkScheduling2000 with the benchmark's own pods (no UID, zero CreationTimestamp; they are never
    applied to an apiserver): NewQueue breaks cpu/memory ties by sort.Slice's swap order over the input
    (queue.go:38, the host's pdqsort emulation) and every pod shares the staleness key "" (queue.go:54-69)."""
    want, got = _solve_both(synth.config1(literal=True))
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", [440, 441, 442, 443])
def test_lean_shared_uids_with_push_backs(seed):
    """Resource-only pods sharing UID "" (BenchmarkScheduling's literal pods) run the LEAN Solve; a pod that
    fails (too large for every instance type, or past a NodePool limit) is pushed back, and the Solve leaves
    the LEAN kernel there (KE_LEAN_EXIT) and re-runs non-LEAN, where Queue.Pop re-reads the shared staleness
    entry (queue.go:54-69).  Seed 440 has no failure (stays LEAN)."""
    snap = synth.benchmark_snapshot(600, 60, seed, diverse=False, literal=True)
    if seed in (441, 443):
        for k in range(3):
            big = synth.pod(900000 + k, cpu="1000", mem="1Gi")
            big["metadata"].pop("uid", None)
            snap["pods"].insert(100 * (k + 1), big)
    if seed in (442, 443):
        pool = synth.node_pool("default-pool", limits={"cpu": "150"})
        snap["nodePools"] = [pool]
    want, got = _solve_both(snap)
    d = _diff(want, got)
    assert d is None, d
    if seed != 440:
        assert want["podErrors"], "the case must push pods back"


@pytest.mark.parametrize("seed", [460, 461, 462, 463, 464])
def test_lean_runs_past_the_queue_window(seed):
    """Resource-only pods with distinct UIDs (the LEAN Solve keeps running after a push-back): long runs of
    identical pods whose NodeClaim runs reach past the 64-pod queue window while nothing has been pushed back
    (run lengths over NewQueue's order, round 6); a pod too large for every instance type (461, 463) or a
    NodePool limit (462, 463) pushes pods back, after which runs stay inside the window; 464 mixes the pods'
    tolerations (same requests, different toleration sets never share a run)."""
    snap = synth.benchmark_snapshot(3000, 60, seed, diverse=False)
    if seed in (461, 463):
        for k in range(3):
            snap["pods"].insert(700 * (k + 1), synth.pod(900000 + k, cpu="1000", mem="1Gi"))
    if seed in (462, 463):
        snap["nodePools"] = [synth.node_pool("default-pool", limits={"cpu": "1500"})]
    if seed == 464:
        for i, p in enumerate(snap["pods"]):
            if i % 3 == 0:
                p["spec"]["tolerations"] = [{"key": "batch", "operator": "Exists"}]
    want, got = _solve_both(snap)
    d = _diff(want, got)
    assert d is None, d
    if seed in (461, 462, 463):
        assert want["podErrors"], "the case must push pods back"


@pytest.mark.parametrize("seed", list(range(400, 412)))
def test_queue_ties_parity(seed):
    """Random problems whose pods share UIDs and timestamps in groups, so NewQueue's order of equal
    (cpu, memory) pods comes from sort.Slice's tie order and staleness is shared per UID."""
    snap = problems.random_problem(seed, n_pods=200, n_nodes=int(seed % 3) * 5)
    for i, p in enumerate(snap["pods"]):
        p["metadata"]["uid"] = "" if seed == 401 else "shared-%d" % (i % 25)
        p["metadata"].pop("creationTimestamp", None)
    want, got = _solve_both(snap)
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", list(range(420, 436)))
def test_same_pod_host_ports_parity(seed):
    """Existing nodes whose HostPortUsage holds entries of the pods being scheduled: Conflicts skips the
    pod's own entries and Add replaces them (hostportusage.go:70-85)."""
    snap = problems.random_problem(seed, n_pods=150, n_nodes=8 + seed % 5, host_ports=True, same_pod_ports=True)
    want, got = _solve_both(snap)
    d = _diff(want, got)
    assert d is None, d
