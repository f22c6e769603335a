"""Production nodes carry dozens of labels no requirement mentions.  The encoder interns an existing node's
label keys only when a requirement, template label or topology key names them (ks_host.cpp universe build):
ExistingNode.Add's strict Compatible reads a node's value of a key only when the pod names it
(existingnode.go:97-104, requirements.go:163-174), and a node's record is never rendered.  So 120 extra
node-only label keys neither hit the 64-key universe cap nor change a result.

CPU: the universe stays under the cap (ks_problem_inspect / ks_cons_inspect).  GPU: Solve and consolidation
equal the oracle, which keeps every label."""
import json

import pytest

import problems
from karpenter_amd import Consolidator, Scheduler, inspect, inspect_consolidation, synth
from oracle import bridge

EXTRA = 120


def _label_nodes(snap, key):
    for i, n in enumerate(snap.get(key, [])):
        labels = n.setdefault("labels", {})
        for k in range(EXTRA):
            labels["example.com/extra-%03d" % k] = "v%d" % ((i + k) % 7)
    return snap


def _solve_snap(seed, topology=False):
    return _label_nodes(problems.random_problem(seed, n_pods=120, n_nodes=16, topology=topology), "stateNodes")


def _cons_snap(seed):
    return _label_nodes(synth.cluster_snapshot(n_nodes=20, pods_per_node=8, n_its=40, seed=seed, n_pending=3,
                                               pod_selectors=True), "stateNodes")


@pytest.mark.parametrize("seed", [70, 71, 72])
def test_node_only_label_keys_stay_out_of_the_universe(seed):
    d = inspect(json.dumps(_solve_snap(seed)))
    assert d["keys"] <= 64 and not any(k.startswith("example.com/extra") for k in d["keyNames"])
    c = inspect_consolidation(json.dumps(_cons_snap(seed)))
    assert c["sims"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("seed,topology", [(70, False), (71, False), (72, True), (73, True)])
def test_solve_with_many_node_labels(seed, topology):
    s = json.dumps(_solve_snap(seed, topology))
    got = Scheduler(s).solve()
    want, _ = bridge.solve(s)
    assert problems.canonical(want) == got.canonical()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [5, 6])
def test_consolidation_with_many_node_labels(seed):
    s = json.dumps(_cons_snap(seed))
    want, _ = bridge.consolidate(s, all_sims=True)
    got = Consolidator(s).consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert got == want
