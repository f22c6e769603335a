"""Cluster-state accounting (pkg/controllers/state): the StateNode accessor values the informers
converge to, derived from Node / NodeClaim / Pod listings.  The oracle (an event replay,
oracle/cluster_state.inc) is pinned by the state suite's assertions (tests/golden/make_state_fixtures.py);
the product's host builder (ks_cluster_state, karpenter-sigs_amd/csrc/ks_state.cpp) must equal the oracle
field by field on those and on random clusters, and its output must feed the consolidation snapshot."""
import json
import os
import random
import re
import sys
from fractions import Fraction

import pytest

from karpenter_amd import cluster_state, inspect_consolidation
from oracle import bridge

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_state_fixtures as msf  # noqa: E402

FIXTURES = json.load(open(os.path.join(HERE, "golden", "state_scenarios.json")))
SCENARIOS = {s["name"]: s for s in msf.scenarios()}
_SUF = {"": 1, "m": Fraction(1, 1000), "k": 1000, "M": 10**6, "G": 10**9, "Ki": 1024, "Mi": 1024**2, "Gi": 1024**3}


def qty(s):
    m = re.fullmatch(r"(-?[0-9.]+)([a-zA-Z]*)", s)
    return Fraction(m.group(1)) * _SUF[m.group(2)]


def host_view(nodes):
    """The host returns each node's bound pods; the oracle reports their count."""
    out = []
    for n in nodes:
        n = dict(n)
        n["podCount"] = len(n.pop("pods"))
        out.append(n)
    return out


@pytest.mark.parametrize("fx", FIXTURES, ids=[f["name"] for f in FIXTURES])
def test_state_scenarios(fx):
    scn = SCENARIOS[fx["name"]]
    assert scn["expect"] == fx["expect"]
    want = bridge.cluster_state(scn["cluster"])
    got = cluster_state(json.dumps(scn["cluster"]))
    assert host_view(got) == want
    assert len(want) == fx["expect"]["count"]
    by = {n["name"]: n for n in want}
    for name, exp in fx["expect"]["nodes"].items():
        n = by[name]
        for field in ("podRequests", "daemonSetRequests"):
            for r, v in exp.get(field, {}).items():  # ExpectResources: missing = 0
                assert qty(n[field].get(r, "0")) == qty(v), (field, r, n[field])
        for drv, cnt in exp.get("volumes", {}).items():  # ExceedsLimits of one more volume: at the limit
            assert len(n["volumeUsage"][drv]) == cnt
        assert n.get("volumeLimits", {}) == exp.get("volumeLimits", n.get("volumeLimits", {}))
        for port in exp.get("hostPorts", []):
            assert any(p["port"] == port for ps in n["hostPortUsage"].values() for p in ps)
        for r, v in n["allocatable"].items():  # Available = Allocatable - PodRequests
            assert qty(n["available"][r]) == qty(v) - qty(n["podRequests"].get(r, "0"))


def random_cluster(seed, n=24):
    """Nodes in every lifecycle state the accessors distinguish: NodeClaim only (launched, not
    registered), registered / initialized pairs, unmanaged nodes (with and without providerID),
    managed nodes without a providerID or an instance-type label, startup and ephemeral taints,
    zero Node resources that the NodeClaim overrides, deletion timestamps; pods bound, unbound,
    terminal, DaemonSet-owned, with host ports, or bound to untracked nodes."""
    rng = random.Random(seed)
    ncs, nodes, pods = [], [], []
    names = []
    eph = [{"key": "node.kubernetes.io/not-ready", "effect": "NoSchedule"},
           {"key": "node.cloudprovider.kubernetes.io/uninitialized", "value": "true", "effect": "NoSchedule"},
           {"key": "node.kubernetes.io/unreachable", "effect": "NoExecute"}]
    for i in range(n):
        name = "node-%02d" % i
        kind = rng.choice(["claim-only", "pair", "pair", "pair-uninit", "unmanaged", "unmanaged-noid",
                           "managed-noid", "managed-noit"])
        cpu, mem = str(rng.choice([2, 4, 8, 16])), "%dGi" % rng.choice([4, 8, 32])
        labels = dict(msf.MANAGED, **{"kubernetes.io/hostname": name} if rng.random() < 0.7 else {})
        taints = [{"key": "team", "value": "a", "effect": "NoSchedule"}] if rng.random() < 0.3 else []
        taints += rng.sample(eph, rng.randint(0, 2))
        startup = [{"key": "example.com/startup", "effect": "NoSchedule"}] if rng.random() < 0.5 else []
        deleting = rng.random() < 0.15
        if kind in ("claim-only", "pair", "pair-uninit"):
            ncs.append(msf.nodeclaim("nc-%02d" % i, "fake:///" + name, labels, {"cpu": cpu, "memory": mem, "pods": "110"},
                                     taints=taints + [{"key": "claim-only", "effect": "NoSchedule"}],
                                     startup_taints=startup, deleting=deleting and rng.random() < 0.5))
        if kind == "claim-only":
            continue
        nl = dict(labels)
        if kind in ("unmanaged", "unmanaged-noid"):
            nl.pop("karpenter.sh/nodepool")
        if kind == "pair":
            nl["karpenter.sh/registered"] = "true"
            if rng.random() < 0.8:
                nl["karpenter.sh/initialized"] = "true"
        if kind == "pair-uninit":
            nl["karpenter.sh/registered"] = rng.choice(["true", "false"])
        if kind == "managed-noit":
            nl.pop("node.kubernetes.io/instance-type")
        alloc = {"cpu": cpu if rng.random() < 0.7 else "0", "memory": mem, "pods": "110"}
        pid = "" if kind in ("unmanaged-noid", "managed-noid") else "fake:///" + name
        nodes.append(msf.node(name, alloc, nl, provider_id=pid, taints=taints + startup, ready=rng.random() < 0.85,
                              capacity={"cpu": cpu, "memory": mem, "pods": "110"}, deleting=deleting))
        names.append(name)
    for j in range(6 * n):
        bound = rng.choice(names + ["", "", "ghost-node"]) if names else ""
        req = {"cpu": rng.choice(["100m", "250m", "1", "1.5"]), "memory": rng.choice(["128Mi", "1Gi", "1.5G"])}
        pods.append(msf.pod("pod-%03d" % j, req, bound, phase=rng.choice(["Running"] * 6 + ["Failed", "Succeeded"]),
                            daemonset=rng.random() < 0.15, host_ports=[8000 + j] if rng.random() < 0.1 else (),
                            ns=rng.choice(["default", "kube-system"]),
                            pvcs=["pvc-%d" % rng.randrange(40)] if rng.random() < 0.3 else ()))
    # PVC -> CSI driver (resolved, "" = no driver, or absent = NotFound) and CSINode limits
    drivers = {}
    for k in range(40):
        for ns in ("default", "kube-system"):
            r = rng.random()
            if r < 0.7:
                drivers["%s/pvc-%d" % (ns, k)] = rng.choice(["ebs.csi", "efs.csi"])
            elif r < 0.85:
                drivers["%s/pvc-%d" % (ns, k)] = ""
    csis = [{"metadata": {"name": nm}, "spec": {"drivers": [
        {"name": "ebs.csi", "allocatable": {"count": rng.randint(1, 30)}},
        {"name": "efs.csi", "allocatable": None}]}} for nm in names if rng.random() < 0.6]
    return {"nodeClaims": ncs, "nodes": nodes, "pods": pods, "volumeDrivers": drivers, "csiNodes": csis}


@pytest.mark.parametrize("seed", range(12))
def test_random_clusters_match_oracle(seed):
    c = random_cluster(seed)
    want = bridge.cluster_state(c)
    got = cluster_state(json.dumps(c))
    assert host_view(got) == want


def consolidatable(c, its, seed):
    """Give the nodes of a random cluster the labels NewCandidate reads (an instance type of the pool,
    its capacity type and zone), and the pods ReplicaSet owners and no host ports (a bound pod holding
    host ports is refused loudly)."""
    rng = random.Random(seed)
    by_name = {}
    for obj in c["nodeClaims"] + c["nodes"]:
        name = obj["metadata"]["name"].replace("nc-", "node-")
        it = by_name.setdefault(name, rng.choice(its))
        off = it["offerings"][0]
        obj["metadata"]["labels"].update({"node.kubernetes.io/instance-type": it["name"],
                                          "karpenter.sh/capacity-type": off["capacityType"],
                                          "topology.kubernetes.io/zone": off["zone"]})
    for p in c["pods"]:
        p["spec"]["containers"][0].pop("ports", None)
        if not p["metadata"].get("ownerReferences"):
            p["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs",
                                                 "uid": "rs-uid"}]
    return c


def test_derived_state_feeds_consolidation():
    """The derived stateNodes are a consolidation snapshot's stateNodes: candidates and costs agree with
    the oracle reading the same snapshot."""
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_consolidation_fixtures as mcf
    its = mcf.assorted()[:64]
    base = mcf.snapshot(its, [])
    c = consolidatable(random_cluster(3, n=16), its, 3)
    state = cluster_state(json.dumps(c))
    base["stateNodes"] = state
    base["candidates"] = [n["name"] for n in state]
    got = inspect_consolidation(json.dumps(base))
    want, _ = bridge.consolidate(json.dumps(base), all_sims=False)
    assert [(x["name"], x["disruptionCost"]) for x in got["candidates"]] == \
        [(x["name"], x["disruptionCost"]) for x in want["candidates"]]
    assert got["candidates"]


def _cons_inputs(seed):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_consolidation_fixtures as mcf
    its = mcf.assorted()[:64]
    c = consolidatable(random_cluster(seed, n=16), its, seed)
    base = mcf.snapshot(its, [])
    base.pop("stateNodes")
    # the oracle reads stateNodes: its own derivation, with each node's bound pods attached in listing order
    state = bridge.cluster_state(c)
    for n in state:
        n["pods"] = [p for p in c["pods"] if n["podCount"] and p["spec"]["nodeName"] == n["name"]]
    with_state = dict(base, stateNodes=state, candidates=[n["name"] for n in state])
    with_cluster = dict(base, cluster=c, candidates=[n["name"] for n in state])
    return with_state, with_cluster


@pytest.mark.parametrize("seed", (5, 6))
def test_consolidation_snapshot_from_listings(seed):
    """ks_cons_create / ks_cons_inspect accept the raw listings ("cluster") in place of "stateNodes"
    and derive the same candidates as the oracle over its own derived state."""
    with_state, with_cluster = _cons_inputs(seed)
    got = inspect_consolidation(json.dumps(with_cluster))
    want, _ = bridge.consolidate(json.dumps(with_state), all_sims=False)
    assert [(x["name"], x["disruptionCost"]) for x in got["candidates"]] == \
        [(x["name"], x["disruptionCost"]) for x in want["candidates"]]
    assert got["candidates"]
