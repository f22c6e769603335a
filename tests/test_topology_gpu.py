"""GPU parity for the Topology path (topology.go / topologygroup.go on k_solve): the HIP Solve vs the
oracle, bit-exact on the canonical Results, over the reference's topology_test.go scenarios
(tests/golden/make_topology_fixtures.py) and seeded random problems with zonal / hostname /
capacity-type spread (maxSkew, minDomains, ScheduleAnyway relaxation, node filters), required and
preferred pod anti-affinity, and bound cluster pods seeding counts and inverse anti-affinity.

PodErrors text is compared verbatim, including a hostname-keyed group's `counts = map[...]` (every
existing node and hostname-placeholder registered so far, topology.go:167)."""
import json
import os
import sys

import pytest

import problems
from karpenter_amd import Scheduler
from oracle import bridge

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_topology_fixtures as mtf  # noqa: E402

pytestmark = pytest.mark.gpu

def _norm(res):
    return problems.canonical(res)


def _solve_both(snap):
    s = json.dumps(snap)
    want, _ = bridge.solve(s)
    got = Scheduler(s).solve().canonical()
    return _norm(want), _norm(got)


def _diff(want, got):
    if want == got:
        return None
    for key in ("newNodeClaims", "existingNodes", "podErrors"):
        if want[key] != got[key]:
            if isinstance(want[key], list):
                for i, (a, b) in enumerate(zip(want[key], got[key])):
                    if a != b:
                        return "%s[%d]: want %s\n got %s" % (key, i, json.dumps(a)[:1500], json.dumps(b)[:1500])
                return "%s: length %d vs %d" % (key, len(want[key]), len(got[key]))
            for k in sorted(set(want[key]) | set(got[key]), key=int):
                if want[key].get(k) != got[key].get(k):
                    return "%s[%s]: want %r\n got %r" % (key, k, want[key].get(k), got[key].get(k))
    return "differs"


SCENARIOS = mtf.scenarios()


@pytest.mark.parametrize("scn", SCENARIOS, ids=[s["name"] for s in SCENARIOS])
def test_reference_topology_scenarios_gpu(scn):
    want, got = _solve_both(scn["snapshot"])
    assert _diff(want, got) is None, _diff(want, got)
    bad = mtf.check(scn, got)
    assert not bad, bad


@pytest.mark.parametrize("seed", list(range(300, 332)))
def test_random_topology_parity(seed):
    want, got = _solve_both(problems.random_problem(seed, n_pods=150, topology=True))
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", list(range(360, 384)))
def test_random_pod_affinity_parity(seed):
    """Required / preferred pod affinity (zone, hostname, capacity-type; to itself or another app)
    mixed with spread and anti-affinity."""
    want, got = _solve_both(problems.random_problem(seed, n_pods=150, topology=True, affinity=True))
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", list(range(390, 406)))
def test_random_namespace_selector_parity(seed):
    """Pods and cluster pods over four namespaces; (anti-)affinity terms with namespace lists and
    namespaceSelectors (empty, by label, with a list) resolved against the snapshot's namespaces."""
    want, got = _solve_both(problems.random_problem(seed, n_pods=150, topology=True, affinity=True, namespaces=True))
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", [340, 341, 342, 343])
def test_random_topology_parity_larger(seed):
    want, got = _solve_both(problems.random_problem(seed, n_pods=800, n_its=120, n_nodes=30, topology=True))
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", [350, 351])
def test_topology_with_host_ports(seed):
    want, got = _solve_both(problems.random_problem(seed, n_pods=200, n_nodes=8, host_ports=True, topology=True))
    d = _diff(want, got)
    assert d is None, d


def test_config4_topology_existing_nodes():
    """C4 shape (BASELINE.json configs[3]) at 2000 pods onto 400 existing nodes with bound cluster
    pods: zonal spread, hostname spread and hostname anti-affinity over 20 apps."""
    from karpenter_amd import synth

    want, got = _solve_both(synth.config4(2000, 400))
    d = _diff(want, got)
    assert d is None, d


def test_config4_full_size_properties():
    """Full C4 (10k pods, 2k nodes): no oracle run at this size; check the invariants the domain
    gives: every pod placed exactly once or failed, and required hostname anti-affinity holds
    against the bound cluster pods and this Solve's own placements."""
    from karpenter_amd import Scheduler, synth

    snap = synth.config4()
    res = Scheduler(json.dumps(snap)).solve()
    node_zone = {n["name"]: n["labels"][synth.ZONE] for n in snap["stateNodes"]}
    seen = {}
    for ni, n in enumerate(res.existing_nodes):
        for p in n["pods"]:
            assert p not in seen
            seen[p] = n["name"]
    for ci, c in enumerate(res.new_nodeclaims):
        for p in c["pods"]:
            assert p not in seen
            seen[p] = "claim-%d" % ci
    assert len(seen) + len(res.pod_errors) == len(snap["pods"])
    host_apps = {}
    for cp in snap["clusterPods"]:
        host_apps.setdefault((cp["metadata"]["labels"]["app"], cp["spec"]["nodeName"]), 0)
        host_apps[(cp["metadata"]["labels"]["app"], cp["spec"]["nodeName"])] += 1
    for p, where in seen.items():
        spec = snap["pods"][p]["spec"]
        app = snap["pods"][p]["metadata"]["labels"]["app"]
        if "affinity" in spec:  # hostname anti-affinity against cluster pods and this Solve's pods
            host_apps[(app, where)] = host_apps.get((app, where), 0) + 1
    for p, where in seen.items():
        if "affinity" in snap["pods"][p]["spec"]:
            app = snap["pods"][p]["metadata"]["labels"]["app"]
            assert host_apps[(app, where)] == 1, (p, where)
    assert all(w in node_zone or w.startswith("claim-") for w in seen.values())


@pytest.mark.parametrize("seed", list(range(440, 456)))
def test_unlabelled_nodes_with_not_in_parity(seed):
    """Existing nodes lacking a topology key's label, with pods admitting them through NotIn /
    DoesNotExist on that key: the node takes the key from the pod's requirements and its domain is
    chosen like a NodeClaim's, then recorded (existingnode.go:91-121); k_solve decides such nodes
    wave-wide (node_slow) and keeps their accumulated requirements."""
    snap = problems.random_problem(seed, n_pods=150, n_nodes=10, topology=True, affinity=seed % 2 == 1)
    problems.unlabel_topology_nodes(snap, seed)
    want, got = _solve_both(snap)
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", list(range(460, 480)))
def test_groups_created_mid_solve_parity(seed):
    """Spread pods with OR'd required node-affinity terms: relaxing term[0] changes the group's node
    filter, so Topology.Update creates a new group mid-Solve (topology.go:102-119) with countDomains over
    the cluster's bound pods only, no hostnames of the existing nodes or earlier NodeClaims registered,
    and no earlier placements recorded."""
    from karpenter_amd import inspect

    snap = problems.random_problem(seed, n_pods=150, n_nodes=int(seed % 3) * 6, topology=True,
                                   affinity=seed % 2 == 1, or_terms=True)
    assert inspect(snap)["lateGroups"] > 0
    want, got = _solve_both(snap)
    d = _diff(want, got)
    assert d is None, d


@pytest.mark.parametrize("seed", list(range(500, 516)))
def test_hostname_topology_errors_parity(seed):
    """Unsatisfiable hostname-keyed pod affinity (problems.hostname_failure_problem): the PodErrors text
    prints the group's registered hostname domains and counts -- existing nodes, every placeholder
    registered so far, this Solve's records (topology.go:167) -- verbatim against the oracle."""
    snap = problems.hostname_failure_problem(seed)
    want, got = _solve_both(snap)
    assert any("key=kubernetes.io/hostname (counts = map[" in v for v in want["podErrors"].values()) or seed in (506, 513, 515)
    d = _diff(want, got)
    assert d is None, d
