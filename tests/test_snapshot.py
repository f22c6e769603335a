"""Binary snapshots of an encoded problem (ks_problem_save / ks_problem_create_binary, ks_cons_save /
ks_cons_create_binary; SURVEY.md §5 "binary problem file").

CPU: the format is the identity through save -> load -> save (ks_snapshot_check) on every shape the suite
encodes (topology, host ports, volumes, limits, taints, the consolidation cluster), and a truncated or
foreign blob is refused.  GPU: a problem / handle rebuilt from its snapshot gives the Results / decisions of
the one built from JSON, and both equal the oracle."""
import json

import pytest

import problems
from karpenter_amd import Consolidator, KsError, Scheduler, snapshot_check, synth
from oracle import bridge

CPU_CASES = ([("random", s) for s in range(6)] + [("topology", s) for s in range(40, 44)] +
             [("hostports", s) for s in range(60, 62)] + [("c1", 0), ("c3", 300), ("c4", 400), ("cluster", 3),
                                                           ("cluster_topo", 4)])


def _snap(kind, arg):
    if kind == "random":
        return problems.random_problem(arg)
    if kind == "topology":
        return problems.random_problem(arg, n_nodes=12, topology=True, affinity=True)
    if kind == "hostports":
        return problems.random_problem(arg, host_ports=True)
    if kind == "c1":
        return synth.config1(literal=True)
    if kind == "c3":
        return synth.config3(arg)
    if kind == "c4":
        return synth.config4(arg, 80)
    if kind == "cluster":
        return synth.cluster_snapshot(n_nodes=20, pods_per_node=8, n_its=40, seed=arg, n_pending=3)
    return synth.cluster_snapshot(n_nodes=30, pods_per_node=6, n_its=40, seed=arg, n_pending=3, topology=8)


@pytest.mark.parametrize("kind,arg", CPU_CASES, ids=["%s-%s" % c for c in CPU_CASES])
def test_snapshot_roundtrip_is_identity(kind, arg):
    n = snapshot_check(json.dumps(_snap(kind, arg)))
    assert n > 0


GPU_SOLVE_CASES = [("random", s) for s in range(4)] + [("topology", 40), ("topology", 41), ("c1", 0), ("c3", 300)]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,arg", GPU_SOLVE_CASES, ids=["%s-%s" % c for c in GPU_SOLVE_CASES])
def test_solve_from_binary_snapshot(kind, arg):
    s = json.dumps(_snap(kind, arg))
    a = Scheduler(s)
    blob = a.save()
    b = Scheduler.from_binary(blob)
    ra, rb = a.solve(), b.solve()
    assert rb.canonical() == ra.canonical()
    want, _ = bridge.solve(s)
    want.pop("stats", None)
    assert problems.canonical(want) == rb.canonical()
    assert b.save() == blob  # the reloaded model saves to the same bytes
    with pytest.raises(KsError):
        Scheduler.from_binary(blob[: len(blob) // 2])
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,topo", [(3, 0), (4, 8), (5, 0)])
def test_consolidation_from_binary_snapshot(seed, topo):
    snap = synth.cluster_snapshot(n_nodes=24, pods_per_node=8, n_its=40, seed=seed, n_pending=3, topology=topo,
                                  spot_frac=0.5)
    s = json.dumps(snap)
    a = Consolidator(s)
    blob = a.save()
    b = Consolidator.from_binary(blob)
    ga, gb = a.consolidate(all_sims=True), b.consolidate(all_sims=True)
    ga.pop("kernel_ms")
    gb.pop("kernel_ms")
    assert gb == ga
    want, _ = bridge.consolidate(s, all_sims=True)
    assert gb == want
    with pytest.raises(KsError):
        Consolidator.from_binary(b"KSPROB01" + blob[8:])  # a problem's magic on a handle's bytes
