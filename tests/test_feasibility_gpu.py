"""k_feasibility (the static pod-state x instance-type rows): k_solve with the rows ANDed in
(the default whenever a pod carries label requirements) and with every key evaluated per step
(KS_NO_FEASIBILITY, read at ks_problem_create) return the same Results, and both equal the oracle.
The rows factor Requirements.Intersects over single-valued keys (requirements.go:241-258); these problems
carry In / NotIn / Exists / DoesNotExist / Gt / Lt terms, OR'd node-affinity terms, preferred terms and
multi-zone offerings, so both factors and the multi-valued remainder are exercised."""
import json
import os

import pytest

import problems
from karpenter_amd import Scheduler, synth
from oracle import bridge

pytestmark = pytest.mark.gpu


def _solve(snap_json, rows):
    if rows:
        os.environ.pop("KS_NO_FEASIBILITY", None)
    else:
        os.environ["KS_NO_FEASIBILITY"] = "1"
    try:
        sch = Scheduler(snap_json)
        r = sch.solve()
        sch.close()
        return r
    finally:
        os.environ.pop("KS_NO_FEASIBILITY", None)


CASES = [("random", s) for s in range(8)] + [("special", s) for s in range(20, 36)] + [("c3", 1500)]


@pytest.mark.parametrize("kind,arg", CASES, ids=["%s-%s" % c for c in CASES])
def test_feasibility_rows_change_nothing(kind, arg):
    """special: NodePool and pod terms on the key some instance types hold as DoesNotExist, where a
    template's Exists meets a pod's NotIn (the row passes DoesNotExist positions; k_solve tests them
    against the whole record's operator)."""
    if kind == "c3":
        snap = synth.config3(arg)
    else:
        snap = problems.random_problem(arg, special=kind == "special")
    s = json.dumps(snap)
    with_rows = _solve(s, True)
    without = _solve(s, False)
    assert with_rows.canonical() == without.canonical()
    want, _ = bridge.solve(s)
    assert problems.canonical(want) == with_rows.canonical()
    if kind == "c3":  # the C3 shape has pods with label requirements: the kernel ran and was timed
        assert with_rows.feasibility_ms > 0 and with_rows.feasibility_bytes > 0
        assert without.feasibility_ms == 0


# --- k_feasibility_nodes: the static pod-state x existing-node rows (taints + strict Compatible) -----------

def _solve_env(snap_json, env):
    """Solve with the given KS_* switches set while the problem is created (ks_problem_create reads them)."""
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update({k: v for k, v in env.items() if v is not None})
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
    try:
        sch = Scheduler(snap_json)
        r = sch.solve()
        sch.close()
        return r
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


NODE_CASES = ([("nodes", s) for s in range(40, 52)] + [("nodes-special", s) for s in range(52, 58)] +
              [("nodes-topology", s) for s in range(58, 64)] + [("nodes-unlabelled", s) for s in range(64, 68)])


@pytest.mark.parametrize("kind,seed", NODE_CASES, ids=["%s-%d" % c for c in NODE_CASES])
def test_node_rows_change_nothing(kind, seed):
    """Existing nodes with taints and labels, pods with selectors / OR'd affinity terms (In, NotIn, Exists,
    DoesNotExist, Gt, Lt): the node scan reading k_feasibility_nodes's bits (and the exact test once a commit
    narrowed a node's requirements, existingnode.go:118) returns the Results of the per-step strict
    Compatible (KS_NO_NODE_ROWS), and both equal the oracle.  nodes-unlabelled: nodes missing a topology
    key's label (decided by node_slow, whose commit replaces the node's record)."""
    snap = problems.random_problem(seed, n_pods=150, n_nodes=16, special=kind == "nodes-special",
                                   topology=kind in ("nodes-topology", "nodes-unlabelled"))
    if kind == "nodes-unlabelled":
        snap = problems.unlabel_topology_nodes(snap, seed)
    s = json.dumps(snap)
    with_rows = _solve_env(s, {"KS_NO_NODE_ROWS": None})
    without = _solve_env(s, {"KS_NO_NODE_ROWS": "1"})
    assert with_rows.canonical() == without.canonical()
    want, _ = bridge.solve(s)
    assert problems.canonical(want) == with_rows.canonical()
    assert without.node_feasibility_ms == 0


def test_node_rows_run_and_are_timed():
    """A problem whose pods carry label requirements onto existing nodes launches k_feasibility_nodes once
    per Solve; its time and algorithmic bytes reach the caller."""
    snap = problems.random_problem(41, n_pods=150, n_nodes=16)
    assert any(p["spec"].get("nodeSelector") or p["spec"].get("affinity") for p in snap["pods"])
    r = _solve_env(json.dumps(snap), {"KS_NO_NODE_ROWS": None})
    assert r.node_feasibility_ms > 0 and r.node_feasibility_bytes > 0


@pytest.mark.parametrize("seed", (5, 24))
def test_node_rows_in_consolidation(seed):
    """Simulations over pods with node selectors: rows on vs off vs the oracle (pod_selectors clusters)."""
    from karpenter_amd import Consolidator
    snap = synth.cluster_snapshot(n_nodes=25, pods_per_node=10, n_its=60, it_range=(8, 30), seed=seed,
                                  pod_selectors=True, topology=3 if seed == 24 else 0)
    s = json.dumps(snap)
    want, _ = bridge.consolidate(s, all_sims=True)
    outs = []
    for env in ({"KS_NO_NODE_ROWS": None}, {"KS_NO_NODE_ROWS": "1"}):
        saved = os.environ.get("KS_NO_NODE_ROWS")
        if env["KS_NO_NODE_ROWS"]:
            os.environ["KS_NO_NODE_ROWS"] = "1"
        else:
            os.environ.pop("KS_NO_NODE_ROWS", None)
        try:
            got = Consolidator(s).consolidate(all_sims=True)
        finally:
            if saved is None:
                os.environ.pop("KS_NO_NODE_ROWS", None)
            else:
                os.environ["KS_NO_NODE_ROWS"] = saved
        got.pop("kernel_ms")
        outs.append(got)
    assert outs[0] == outs[1]
    assert outs[0] == want
