"""Incremental consolidation updates (ks_cons_update).

Between two disruption passes the cluster changes: pods are deleted, pending pods get bound, nodes go away
(state/cluster.go:220-512).  The reference re-reads the cluster and rebuilds its scheduler for every
simulation (provisioner.go:204-296); the resident handle applies the events instead.  The check is always
against a from-scratch build of the snapshot the events lead to (tests/cons_delta.apply_delta edits the
JSON independently of the C++ update):
  CPU: the host half (candidates, costs and order, pending pods, every active node's encoded available row
       and pods, pool limits, simulation plan) equals the from-scratch encode after a sequence of deltas;
       invalid deltas are refused whole; the binary snapshot of an updated handle round-trips.
  GPU: after every delta of a sequence, a pass on the updated handle equals the oracle's consolidation of
       the edited snapshot (every simulation's outcome and both commands), also through save/from_binary.
"""
import json
import random

import pytest

from cons_delta import apply_delta, delta_sequence
from karpenter_amd import Consolidator, KsError, inspect_consolidation_update, synth
from oracle import bridge

SEEDS = [1, 2, 3, 4]


def _snap(seed, n_nodes=40, pods_per_node=5, n_pending=8, pdbs=True):
    return synth.cluster_snapshot(n_nodes=n_nodes, pods_per_node=pods_per_node, n_its=40, seed=seed,
                                  n_pending=n_pending, pdbs=pdbs, limits={"cpu": "2000"} if seed % 2 else None)


@pytest.mark.parametrize("seed", SEEDS)
def test_update_sequence_host_state(seed):
    snap = _snap(seed)
    deltas, final = delta_sequence(seed, snap, steps=4)
    got = inspect_consolidation_update(json.dumps(snap), deltas)
    want = inspect_consolidation_update(json.dumps(final))
    for k in ("candidates", "pendingPods", "nodeRows", "poolRemaining", "sims", "multiPrefixes", "resources"):
        assert got[k] == want[k], k
    # the deltas did move the state
    before = inspect_consolidation_update(json.dumps(snap))
    assert before["nodeRows"] != got["nodeRows"] and before["pendingPods"] != got["pendingPods"]


def test_update_each_kind_alone():
    snap = _snap(7)
    node = snap["stateNodes"][3]
    pend = snap["pendingPods"][0]["metadata"]["uid"]
    for d in ({"deletePods": [node["pods"][0]["metadata"]["uid"]]},
              {"deletePods": [pend]},
              {"bindPods": [{"uid": pend, "node": node["name"]}]},
              {"removeNodes": [node["name"]]},
              {"removeNodes": [snap["stateNodes"][0]["name"], snap["stateNodes"][-1]["name"]]},
              # bound to a node that is removed in the same update: the pod leaves with it
              {"bindPods": [{"uid": pend, "node": node["name"]}], "removeNodes": [node["name"]]},
              # every pod of a node deleted: an empty candidate (cost 0) leads the order
              {"deletePods": [p["metadata"]["uid"] for p in node["pods"]]}):
        got = inspect_consolidation_update(json.dumps(snap), d)
        want = inspect_consolidation_update(json.dumps(apply_delta(snap, d)))
        for k in ("candidates", "pendingPods", "nodeRows", "poolRemaining", "sims"):
            assert got[k] == want[k], (d, k)


def test_bind_unblocks_and_blocks():
    # a do-not-disrupt pending pod bound to a candidate takes that candidate out of the pass
    snap = _snap(8, pdbs=False)
    p = snap["pendingPods"][0]
    p["metadata"]["annotations"] = {"karpenter.sh/do-not-disrupt": "true"}
    target = snap["stateNodes"][5]["name"]
    d = {"bindPods": [{"uid": p["metadata"]["uid"], "node": target}]}
    got = inspect_consolidation_update(json.dumps(snap), d)
    assert target not in [c["name"] for c in got["candidates"]]
    assert got["candidates"] == inspect_consolidation_update(json.dumps(apply_delta(snap, d)))["candidates"]
    # deleting it again brings the candidate back
    d2 = {"deletePods": [p["metadata"]["uid"]]}
    got2 = inspect_consolidation_update(json.dumps(snap), [d, d2])
    assert target in [c["name"] for c in got2["candidates"]]


@pytest.mark.parametrize("bad,code", [
    ({"deletePods": ["no-such-pod"]}, "KS_ERR_ARG"),
    ({"bindPods": [{"uid": "pod-uid-000000", "node": "node-00001"}]}, "KS_ERR_ARG"),  # bound, not pending
    ({"removeNodes": ["node-99999"]}, "KS_ERR_ARG"),
    ({"removeNodes": ["node-00001", "node-00001"]}, "KS_ERR_ARG"),
    ({"deletePods": ["pod-uid-000000", "pod-uid-000000"]}, "KS_ERR_ARG"),
    ({"evictPods": []}, "KS_ERR_PARSE"),
])
def test_invalid_updates_are_refused(bad, code):
    snap = _snap(9)
    with pytest.raises(KsError) as e:
        inspect_consolidation_update(json.dumps(snap), bad)
    assert code in str(e.value)
    # a sequence stops at the refused delta
    with pytest.raises(KsError):
        inspect_consolidation_update(json.dumps(snap), [{"deletePods": ["pod-uid-000001"]}, bad])


def _topo_snap(seed, apps=8):
    return synth.cluster_snapshot(n_nodes=30, pods_per_node=5, n_its=40, seed=seed, n_pending=6, topology=apps)


def _owned_topology(doc):
    return {k: (v["late"], v["counts"]) for k, v in doc["topology"].items() if v["owned"]}


@pytest.mark.parametrize("seed", [21, 22, 23])
def test_topology_update_host_state(seed):
    """Topology clusters: after a delta sequence the shared NewTopology counts of every group a remaining pod
    owns equal a from-scratch build's (registered domains and counts, late flag); groups only the updated
    handle holds are owned by no pod."""
    snap = _topo_snap(seed)
    deltas, final = delta_sequence(seed, snap, steps=4, n_del=4, n_bind=3)
    got = inspect_consolidation_update(json.dumps(snap), deltas)
    want = inspect_consolidation_update(json.dumps(final))
    for k in ("candidates", "pendingPods", "nodeRows", "poolRemaining", "sims"):
        assert got[k] == want[k], k
    assert _owned_topology(got) == _owned_topology(want)
    before = inspect_consolidation_update(json.dumps(snap))
    assert _owned_topology(before) != _owned_topology(got)


def test_topology_update_each_kind_alone():
    snap = _topo_snap(24)
    node = snap["stateNodes"][2]
    pend = snap["pendingPods"][0]["metadata"]["uid"]
    for d in ({"deletePods": [node["pods"][0]["metadata"]["uid"]]},
              {"bindPods": [{"uid": pend, "node": node["name"]}]},
              {"removeNodes": [node["name"]]},
              {"bindPods": [{"uid": pend, "node": node["name"]}], "removeNodes": [node["name"]]},
              {"deletePods": [p["metadata"]["uid"] for p in node["pods"]]}):
        got = inspect_consolidation_update(json.dumps(snap), d)
        want = inspect_consolidation_update(json.dumps(apply_delta(snap, d)))
        assert _owned_topology(got) == _owned_topology(want), d
        assert got["sims"] == want["sims"] and got["candidates"] == want["candidates"], d


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_update_sequence_gpu_parity(seed):
    snap = _snap(seed)
    deltas, _ = delta_sequence(seed, snap, steps=4)
    c = Consolidator(json.dumps(snap))
    # all or nothing: a refused delta (its first events valid) leaves the handle as it was
    with pytest.raises(KsError):
        c.update({"deletePods": [deltas[0]["deletePods"][0]], "removeNodes": ["node-99999"]})
    want, _ = bridge.consolidate(json.dumps(snap), all_sims=True)
    got = c.consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert got == want
    cur = snap
    for i, d in enumerate(deltas):
        c.update(d)
        cur = apply_delta(cur, d)
        want, _ = bridge.consolidate(json.dumps(cur), all_sims=True)
        got = c.consolidate(all_sims=True)
        got.pop("kernel_ms")
        assert got == want, (seed, i)
    # the updated handle's binary snapshot is the updated cluster
    c2 = Consolidator.from_binary(c.save())
    got = c2.consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert got == want
    # and updates continue from a loaded handle
    d, _ = delta_sequence(seed + 100, cur, steps=1)
    c2.update(d[0])
    want, _ = bridge.consolidate(json.dumps(apply_delta(cur, d[0])), all_sims=True)
    got = c2.consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [31, 32, 33])
def test_topology_update_sequence_gpu_parity(seed):
    """a topology cluster's handle follows deltas (shared counts re-uploaded); every pass
    equals the oracle's consolidation of the edited snapshot."""
    snap = _topo_snap(seed)
    deltas, _ = delta_sequence(seed, snap, steps=3, n_del=4, n_bind=3)
    c = Consolidator(json.dumps(snap))
    cur = snap
    for i, d in enumerate(deltas):
        c.update(d)
        cur = apply_delta(cur, d)
        want, _ = bridge.consolidate(json.dumps(cur), all_sims=True)
        got = c.consolidate(all_sims=True)
        got.pop("kernel_ms")
        assert got == want, (seed, i)
    c2 = Consolidator.from_binary(c.save())
    got = c2.consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12])
def test_update_then_validate_gpu(seed):
    """Validation after the wait (validation.go:68-180) against an updated handle == the oracle's
    validation against the edited snapshot, for the pass's commands and single-node replacements."""
    snap = _snap(seed)
    c = Consolidator(json.dumps(snap))
    doc = c.consolidate(all_sims=True)
    cmds = [doc["multi"]["command"], doc["single"]["command"]]
    for sim in doc["single"]["sims"][:6]:
        cmd = {"action": "replace", "candidates": sim["candidates"]}
        if sim.get("claim0"):
            cmd["replacement"] = {"instanceTypeOptions": sim["claim0"]["instanceTypeOptions"][:5]}
        cmds.append(cmd)
    deltas, cur = delta_sequence(seed, snap, steps=2, n_rm=2)
    for d in deltas:
        c.update(d)
    for cmd in cmds:
        want = bridge.validate(cur, cmd)
        got = c.validate(cmd)
        assert got == want, cmd


def _ports_snap(seed):
    """Bound pods holding host ports (their nodes' HostPortUsage lists them under the pod's key) and pending pods
    asking for the same ports: a deleted holder frees its port on that node."""
    rng = random.Random(seed)
    snap = _snap(seed, n_nodes=24, pods_per_node=4, n_pending=6, pdbs=False)
    ports = [8080, 9090]
    holders = []
    for n in snap["stateNodes"]:
        for p in n.get("pods", []):
            if rng.random() < 0.5:
                port = rng.choice(ports)
                p["spec"]["containers"][0]["ports"] = [{"containerPort": port, "hostPort": port, "protocol": "TCP"}]
                n.setdefault("hostPortUsage", {})["default/" + p["metadata"]["name"]] = [
                    {"ip": "0.0.0.0", "port": port, "protocol": "TCP"}]
                holders.append(p["metadata"]["uid"])
    for p in snap["pendingPods"][:4]:
        port = rng.choice(ports)
        p["spec"]["containers"][0]["ports"] = [{"containerPort": port, "hostPort": port, "protocol": "TCP"}]
    return snap, holders


@pytest.mark.parametrize("seed", [41, 42])
def test_host_port_pod_deletion_host_state(seed):
    """Deleting pods that hold host ports (round 6: HostPortUsage.DeletePod on the node's mask); binding one is
    still refused (its entries would need host-port classes of their own)."""
    snap, holders = _ports_snap(seed)
    d = {"deletePods": holders[:5], "removeNodes": [snap["stateNodes"][-1]["name"]]}
    got = inspect_consolidation_update(json.dumps(snap), d)
    want = inspect_consolidation_update(json.dumps(apply_delta(snap, d)))
    for k in ("candidates", "pendingPods", "nodeRows", "poolRemaining", "sims"):
        assert got[k] == want[k], k
    with pytest.raises(KsError) as e:
        inspect_consolidation_update(json.dumps(snap), {"bindPods": [
            {"uid": snap["pendingPods"][0]["metadata"]["uid"], "node": snap["stateNodes"][0]["name"]}]})
    assert "KS_ERR_UNSUPPORTED" in str(e.value)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [41, 42, 43])
def test_host_port_pod_deletion_gpu_parity(seed):
    """After deleting host-port holders (and binding port-less pods), a pass on the updated handle equals the
    oracle's consolidation of the edited snapshot, where the deleted pods' entries left their nodes."""
    snap, holders = _ports_snap(seed)
    c = Consolidator(json.dumps(snap))
    plain = [p["metadata"]["uid"] for p in snap["pendingPods"][4:]]
    cur = snap
    for d in ({"deletePods": holders[:4]},
              {"deletePods": holders[4:8], "bindPods": [{"uid": plain[0], "node": snap["stateNodes"][1]["name"]}]},
              {"deletePods": holders[8:10], "removeNodes": [snap["stateNodes"][2]["name"]]}):
        c.update(d)
        cur = apply_delta(cur, d)
        want, _ = bridge.consolidate(json.dumps(cur), all_sims=True)
        got = c.consolidate(all_sims=True)
        got.pop("kernel_ms")
        assert got == want, d
    c2 = Consolidator.from_binary(c.save())
    got = c2.consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert got == want


def _mounts(pod):
    return any(v.get("persistentVolumeClaim") or v.get("ephemeral") for v in pod["spec"].get("volumes", []))


def _volume_delta(snap, seed):
    """Events that leave every node's VolumeUsage as it is: volume-free pods deleted and bound, a node removed
    (with its pods, volumes or not)."""
    rng = random.Random(seed)
    nodes = snap["stateNodes"]
    free = [p["metadata"]["uid"] for n in nodes[:-1] for p in n.get("pods", []) if not _mounts(p)]
    pend = [p["metadata"]["uid"] for p in snap.get("pendingPods", []) if not _mounts(p)]
    d = {"deletePods": rng.sample(free, min(4, len(free))), "removeNodes": [nodes[-1]["name"]]}
    if pend:
        d["bindPods"] = [{"uid": pend[0], "node": nodes[1]["name"]}]
    return d


@pytest.mark.parametrize("seed", [71, 72])
def test_volume_cluster_update_host_state(seed):
    """Clusters with volume limits take updates whose pods mount no volumes (round 6); a pod that mounts one is
    refused (a snapshot reports a node's VolumeUsage as one union per driver, so its share is not known)."""
    from test_volume_topology import _volume_cluster

    snap = _volume_cluster(seed, n_nodes=24, ppn=10)
    d = _volume_delta(snap, seed)
    assert d["deletePods"], "the cluster must hold volume-free pods"
    got = inspect_consolidation_update(json.dumps(snap), d)
    want = inspect_consolidation_update(json.dumps(apply_delta(snap, d)))
    for k in ("candidates", "pendingPods", "nodeRows", "poolRemaining", "sims"):
        assert got[k] == want[k], k
    vol = [p["metadata"]["uid"] for n in snap["stateNodes"] for p in n.get("pods", []) if _mounts(p)]
    with pytest.raises(KsError) as e:
        inspect_consolidation_update(json.dumps(snap), {"deletePods": vol[:1]})
    assert "KS_ERR_UNSUPPORTED" in str(e.value)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [71, 72, 73])
def test_volume_cluster_update_gpu_parity(seed):
    """A pass on the updated handle of a volume-limit cluster equals the oracle's consolidation of the edited
    snapshot, over two successive updates and through save/from_binary."""
    from test_volume_topology import _volume_cluster

    snap = _volume_cluster(seed, n_nodes=24, ppn=10)
    c = Consolidator(json.dumps(snap))
    cur = snap
    for i in range(2):
        d = _volume_delta(cur, seed + i)
        c.update(d)
        cur = apply_delta(cur, d)
        want, _ = bridge.consolidate(json.dumps(cur), all_sims=True)
        got = c.consolidate(all_sims=True)
        got.pop("kernel_ms")
        assert got == want, (seed, i)
    c2 = Consolidator.from_binary(c.save())
    got = c2.consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert got == want


def _late_snap():
    """Pod A's first state owns a zonal spread group whose node filter is term T2; pod B's first state has
    required node-affinity terms [T1, T2] (another group), and its relaxation (removeRequiredNodeAffinityTerm,
    preferences.go:75-89) leaves [T2]: A's group."""
    snap = synth.cluster_snapshot(n_nodes=6, pods_per_node=3, n_its=40, seed=5, n_pending=2)
    t1 = {"matchExpressions": [{"key": "kubernetes.io/arch", "operator": "In", "values": ["arm64"]}]}
    t2 = {"matchExpressions": [{"key": "kubernetes.io/os", "operator": "In", "values": ["linux"]}]}
    spread = [{"maxSkew": 1, "topologyKey": "topology.kubernetes.io/zone", "whenUnsatisfiable": "DoNotSchedule",
               "labelSelector": {"matchLabels": {"app": "x"}}},
              {"maxSkew": 1, "topologyKey": "kubernetes.io/hostname", "whenUnsatisfiable": "DoNotSchedule",
               "labelSelector": {"matchLabels": {"app": "x"}}}]
    a, b = snap["stateNodes"][0]["pods"][0], snap["stateNodes"][1]["pods"][0]
    for p, terms in ((a, [t2]), (b, [t1, t2])):
        p["metadata"]["labels"]["app"] = "x"
        p["spec"]["topologySpreadConstraints"] = spread
        p["spec"]["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
            "nodeSelectorTerms": terms}}}
    snap["clusterPods"] = [p for n in snap["stateNodes"] for p in n["pods"]]
    return snap, a, b


def test_topology_update_turns_a_group_late():
    """Deleting A leaves A's groups owned only by B's relaxed state: a fresh build of the edited cluster creates
    them mid-Solve (late: no node hostname registered).  The update turns them late the same way (round 5
    refused it); deleting B instead changes no group's form."""
    snap, a, b = _late_snap()
    base = inspect_consolidation_update(json.dumps(snap))
    assert base["groups"] >= 4
    for p in (a, b):
        d = {"deletePods": [p["metadata"]["uid"]]}
        got = inspect_consolidation_update(json.dumps(snap), d)
        want = inspect_consolidation_update(json.dumps(apply_delta(snap, d)))
        assert _owned_topology(got) == _owned_topology(want)
        if p is a:
            assert any(late for late, _ in _owned_topology(want).values())


@pytest.mark.gpu
def test_topology_update_turns_a_group_late_gpu():
    snap, a, _ = _late_snap()
    d = {"deletePods": [a["metadata"]["uid"]]}
    c = Consolidator(json.dumps(snap))
    c.update(d)
    want, _ = bridge.consolidate(json.dumps(apply_delta(snap, d)), all_sims=True)
    got = c.consolidate(all_sims=True)
    got.pop("kernel_ms")
    assert got == want
