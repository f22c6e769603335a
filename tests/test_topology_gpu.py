"""GPU parity for the Topology path (topology.go / topologygroup.go on k_solve): the HIP Solve vs the
oracle, bit-exact on the canonical Results, over the reference's topology_test.go scenarios
(tests/golden/make_topology_fixtures.py) and seeded random problems with zonal / hostname /
capacity-type spread (maxSkew, minDomains, ScheduleAnyway relaxation, node filters), required and
preferred pod anti-affinity, and bound cluster pods seeding counts and inverse anti-affinity.

One message detail is normalised on both sides: for a hostname-keyed group the failure text's
`counts = map[...]` lists every NodeClaim placeholder registered so far, which the device does not
snapshot (Topology).  Everything else in the text is compared verbatim."""
import json
import os
import re
import sys

import pytest

import problems
from karpenter_amd import Scheduler
from oracle import bridge

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_topology_fixtures as mtf  # noqa: E402

pytestmark = pytest.mark.gpu

_HOST_COUNTS = re.compile(r"(key=kubernetes\.io/hostname \(counts = )map\[[^\]]*\]")


def _norm(res):
    d = problems.canonical(res)
    d["podErrors"] = {k: _HOST_COUNTS.sub(r"\1map[<hostname counts>]", v) for k, v in d["podErrors"].items()}
    return d


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
