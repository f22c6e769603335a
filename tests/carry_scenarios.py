"""Constructed clusters where multi-node consolidation's probes share mutated candidate pods.

The reference's binary search (multinodeconsolidation.go:101-135) re-uses the Candidate.pods objects that
NewCandidate listed once per pass (types.go:114-126): each probe appends the same *v1.Pod pointers to its
simulation (helpers.go:102-104) and its Solve relaxes them in place (preferences.go:60-147).  A pod one probe
relaxed therefore starts the next probe relaxed: it is not pushed to the back of the queue first, and the
topology groups its dropped constraints implied are not created for it.

Layout of every scenario (4 candidates, so the search probes mid = 2, then mid = 1 when that fails):
  cand-0  P: 3 cpu, a constraint its first relaxation state can never satisfy (which), so probe 1 relaxes it
  cand-1  R: 2 cpu
  cand-2  X: 100 cpu, fits no instance type -> probe 1 (candidates 0-2) is a no-op
  cand-3  Y: 1 cpu
  keep-1 (3 cpu free) and keep-2 (2 cpu free): non-candidate nodes

Probe 2 (candidates 0-1) with the carried P: P (queued first, 3 cpu) fills keep-1, R fills keep-2, so the
command deletes both.  From pristine pods, P fails its first state, goes to the back of the queue, R takes
keep-1 first and P needs a new NodeClaim: a replacement.  The first-state constraint `which`:
  pref-node     preferred node affinity to a zone no node or instance type has
  pref-pod      preferred zonal pod affinity to an app no pod runs
  pref-anti     preferred zonal pod anti-affinity to an app running in the only zone
  pref-node-2   two impossible preferred node-affinity terms (two relaxations)
  spread-any    ScheduleAnyway zonal spread with minDomains above the zone count (see make())
  pns           a PreferNoSchedule taint on the keep nodes and the template; P's first state does not tolerate it
  late-carry    an impossible first required node-affinity term and a hostname spread (see make())
Variant 1 gives keep-1 room for P and R together: there the carried and the pristine probe agree.
"""
import copy
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
sys.path.insert(0, os.path.join(HERE, "..", "karpenter-sigs_amd"))
import make_consolidation_fixtures as mcf  # noqa: E402
from karpenter_amd import synth  # noqa: E402

KINDS = ["pref-node", "pref-pod", "pref-anti", "pref-node-2", "spread-any", "pns", "late-carry"]


def _its():
    big = synth.fake_instance_type("big-8", 8, 16, pods=20, offerings=[
        {"capacityType": "on-demand", "zone": "test-zone-1", "price": 2.0, "available": True}])
    small = synth.fake_instance_type("small-4", 4, 8, pods=20, offerings=[
        {"capacityType": "on-demand", "zone": "test-zone-1", "price": 0.1, "available": True}])
    return [big, small]


def _bound(pod, node):
    pod["spec"]["nodeName"] = node
    pod["status"] = {"phase": "Running", "conditions": [{"type": "PodScheduled", "status": "True"}]}
    pod["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs", "uid": "rs-uid"}]
    return pod


def make(which, variant=0, volumes=False):
    """One constructed cluster snapshot; `variant` shifts the keep nodes' free capacity (variant 1: keep-1 has
    room for P and R together, so carried and pristine agree: the control case).  volumes: P mounts a claim bound
    to a PV whose node affinity is the one zone, so VolumeTopology.Inject adds that zone to P's required terms in
    every probe (volumetopology.go:41-77)."""
    its = _its()
    big, small = its
    zone_aff = None
    p_extra = {}
    p_labels = {"app": "p"}
    if which == "pref-node":
        zone_aff = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 10, "preference": {"matchExpressions": [
                {"key": synth.ZONE, "operator": "In", "values": ["nowhere"]}]}}]}}
    elif which == "pref-node-2":  # two preferred terms: two relaxations, both impossible
        zone_aff = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 5, "preference": {"matchExpressions": [
                {"key": synth.ZONE, "operator": "In", "values": ["nowhere-b"]}]}},
            {"weight": 10, "preference": {"matchExpressions": [
                {"key": synth.ZONE, "operator": "In", "values": ["nowhere"]}]}}]}}
    elif which == "pref-pod":
        zone_aff = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 10, "podAffinityTerm": {"topologyKey": synth.ZONE,
                                               "labelSelector": {"matchLabels": {"app": "ghost"}}}}]}}
    elif which == "pref-anti":  # zonal anti-affinity to app q, which runs on every keep node's zone
        zone_aff = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
            {"weight": 10, "podAffinityTerm": {"topologyKey": synth.ZONE,
                                               "labelSelector": {"matchLabels": {"app": "q"}}}}]}}
    elif which == "spread-any":
        # zonal spread over app=p, ScheduleAnyway, maxSkew 1, minDomains 3: the one zone already holds two app=p
        # pods (keep-1's fillers) and fewer domains than minDomains put the global minimum at 0
        # (topologygroup.go:194-212), so 2 + 1 - 0 > 1 everywhere until the constraint is relaxed away
        p_extra = {"topologySpreadConstraints": [
            {"maxSkew": 1, "topologyKey": synth.ZONE, "whenUnsatisfiable": "ScheduleAnyway", "minDomains": 3,
             "labelSelector": {"matchLabels": {"app": "p"}}}]}
    elif which == "pns":
        pass
    elif which == "late-carry":
        # two required node-affinity terms, the first matching nothing, and a hostname spread: the state after
        # the term is dropped owns a spread group no pod's first state creates (a late group of the problem,
        # ks_topo.cpp), which a probe starting P in that state creates at NewTopology time, with every existing
        # node's hostname registered
        zone_aff = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
            {"matchExpressions": [{"key": synth.ZONE, "operator": "In", "values": ["nowhere"]}]},
            {"matchExpressions": [{"key": synth.ZONE, "operator": "In", "values": ["test-zone-1"]}]}]}}}
        p_extra = {"topologySpreadConstraints": [
            {"maxSkew": 1, "topologyKey": synth.HOSTNAME, "whenUnsatisfiable": "DoNotSchedule",
             "labelSelector": {"matchLabels": {"app": "p"}}}]}
    else:
        raise ValueError(which)
    P = synth.pod(1, cpu="3", labels=p_labels, affinity=zone_aff, extra=p_extra or None)
    R = synth.pod(2, cpu="2", labels={"app": "r"}, tolerations=[  # (pns: R tolerates the soft taint from the start)
        {"key": "soft", "operator": "Exists", "effect": "PreferNoSchedule"}] if which == "pns" else None)
    X = synth.pod(3, cpu="100", labels={"app": "x"})
    Y = synth.pod(4, cpu="1", labels={"app": "y"})
    for pod, prio in ((P, 0), (R, 1), (X, 2), (Y, 3)):  # disruption cost order: cand-0 .. cand-3
        if prio:
            pod["spec"]["priority"] = prio
    cands = []
    for i, pod in enumerate((P, R, X, Y)):  # each candidate full: no pod of another fits there
        name = "cand-%d" % i
        cpu = pod["spec"]["containers"][0]["resources"]["requests"]["cpu"]
        cands.append(mcf.node(name, big, {"cpu": cpu, "pods": "20"}, [_bound(pod, name)]))
    # keep nodes: free cpu (3, 2) (variant 1: (5, 2)); fillers of app q (pref-anti) or app p (spread-any)
    free1 = 5 if variant == 1 else 3
    fill_app = "p" if which == "spread-any" else "q"
    f1 = [_bound(synth.pod(10, cpu="%d" % (4 - free1) if free1 < 4 else "500m", labels={"app": fill_app}), "keep-1")]
    if which == "spread-any":
        f1.append(_bound(synth.pod(11, cpu="100m", labels={"app": fill_app}), "keep-1"))
    alloc1 = {"cpu": "4" if free1 < 4 else "5.5", "pods": "20"}
    keep1 = mcf.node("keep-1", small, alloc1, f1)
    keep2 = mcf.node("keep-2", small, {"cpu": "4", "pods": "20"},
                     [_bound(synth.pod(12, cpu="2", labels={"app": "q"}), "keep-2")])
    nodes = cands + [keep1, keep2]
    snap = mcf.snapshot(its, nodes)
    snap["candidates"] = [n["name"] for n in cands]
    if which == "pns":
        np_ = snap["nodePools"][0]
        np_["spec"]["template"]["spec"]["taints"] = [{"key": "soft", "value": "x", "effect": "PreferNoSchedule"}]
        snap["nodeClaimTemplates"] = [np_]
        for k in (keep1, keep2):
            k["taints"] = [{"key": "soft", "value": "x", "effect": "PreferNoSchedule"}]
    if volumes:
        P["spec"]["volumes"] = [{"name": "data", "persistentVolumeClaim": {"claimName": "data-p"}}]
        snap["persistentVolumeClaims"] = [{"metadata": {"name": "data-p", "namespace": "default"},
                                           "spec": {"volumeName": "pv-data-p", "storageClassName": ""}}]
        snap["persistentVolumes"] = [{"metadata": {"name": "pv-data-p"}, "spec": {
            "csi": {"driver": "ebs.csi.aws.com", "volumeHandle": "h"},
            "nodeAffinity": {"required": {"nodeSelectorTerms": [{"matchExpressions": [
                {"key": synth.ZONE, "operator": "In", "values": ["test-zone-1"]}]}]}}}}]
        snap["storageClasses"] = []
    # every bound pod is in clusterPods (NewTopology's countDomains source)
    snap["clusterPods"] = [copy.deepcopy(p) for n in nodes for p in n["pods"]]
    return snap


def all_snapshots():
    out = []
    for k in KINDS:
        for v in (0, 1):
            out.append(("%s-v%d" % (k, v), make(k, v)))
    return out


def random_cluster(seed, n_cands=12, n_keep=4, topology=True):
    """A random cluster whose candidate pods carry constraints their first relaxation states often cannot meet
    (the kinds above, mixed), with tight keep nodes: multi-node probes relax pods that later probes hold."""
    import numpy as np

    rng = np.random.default_rng(seed)
    its = _its()
    big, small = its
    soft = [None, "pref-node", "pref-pod", "pref-anti", "pref-node-2", "spread-any"]
    nodes, uid = [], [100]

    def mk(cpu, kind, app):
        uid[0] += 1
        aff, extra = None, None
        if kind == "pref-node":
            aff = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": int(rng.integers(1, 20)), "preference": {"matchExpressions": [
                    {"key": synth.ZONE, "operator": "In", "values": ["nowhere"]}]}}]}}
        elif kind == "pref-node-2":
            aff = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 5, "preference": {"matchExpressions": [
                    {"key": synth.ZONE, "operator": "In", "values": ["test-zone-1"]}]}},
                {"weight": 10, "preference": {"matchExpressions": [
                    {"key": synth.ZONE, "operator": "In", "values": ["nowhere"]}]}}]}}
        elif kind == "pref-pod":
            aff = {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 10, "podAffinityTerm": {"topologyKey": synth.ZONE if rng.random() < 0.5 else synth.HOSTNAME,
                                                   "labelSelector": {"matchLabels": {"app": "ghost" if rng.random() < 0.6 else "a%d" % int(rng.integers(3))}}}}]}}
        elif kind == "pref-anti":
            aff = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 10, "podAffinityTerm": {"topologyKey": synth.HOSTNAME if rng.random() < 0.5 else synth.ZONE,
                                                   "labelSelector": {"matchLabels": {"app": "a%d" % int(rng.integers(3))}}}}]}}
        elif kind == "spread-any":
            extra = {"topologySpreadConstraints": [
                {"maxSkew": 1, "topologyKey": synth.HOSTNAME if rng.random() < 0.5 else synth.ZONE,
                 "whenUnsatisfiable": "ScheduleAnyway",
                 **({"minDomains": 3} if rng.random() < 0.5 else {}),
                 "labelSelector": {"matchLabels": {"app": app}}}]}
        p = synth.pod(uid[0], cpu="%dm" % cpu, labels={"app": app}, affinity=aff, extra=extra)
        if rng.random() < 0.3:
            p["spec"]["priority"] = int(rng.integers(1, 5))
        return p

    for i in range(n_cands):
        name = "cand-%02d" % i
        pods = []
        for _ in range(int(rng.integers(1, 4))):
            kind = soft[int(rng.integers(len(soft)))] if topology or rng.random() < 0.5 else None
            if not topology and kind not in (None, "pref-node", "pref-node-2"):
                kind = "pref-node"
            pods.append(_bound(mk(int(rng.choice([250, 500, 1000, 1500, 2000, 3000])), kind, "a%d" % int(rng.integers(3))),
                               name))
        if rng.random() < 0.15:  # an unschedulable pod: probes holding this candidate fail
            pods.append(_bound(mk(100000, None, "x"), name))
        used = sum(int(p["spec"]["containers"][0]["resources"]["requests"]["cpu"][:-1]) for p in pods)
        nodes.append(mcf.node(name, big, {"cpu": "%g" % (used / 1000.0), "pods": "20"}, pods))
    for k in range(n_keep):
        name = "keep-%d" % k
        fill = int(rng.integers(500, 3500))
        pods = [_bound(mk(fill, None, "a%d" % int(rng.integers(3))), name)]
        nodes.append(mcf.node(name, small, {"cpu": "4", "pods": "20"}, pods))
    snap = mcf.snapshot(its, nodes)
    snap["candidates"] = [n["name"] for n in nodes if n["name"].startswith("cand")]
    if topology:
        snap["clusterPods"] = [copy.deepcopy(p) for n in nodes for p in n["pods"]]
    return snap


def late_group_cluster(variant=0):
    """A group the whole problem creates at NewTopology time (pod A's first state owns it) but one simulation
    creates only mid-Solve: pod B's first state holds an extra required node-affinity term (no node or instance
    type matches it) ahead of A's, so its spread group's node filter differs (topologynodefilter.go:33-51); the
    relaxation that drops the term (preferences.go:75-89) leaves B owning A's group.  In B's single-node
    simulation A is a bound pod on a node that stays, so that group is created by Topology.Update after the
    relaxation (topology.go:102-119): with no hostname registered for the nodes that run no app=w pod
    (existingnode.go:60 ran before it existed), B can take no existing node.  Variant 1 gives A no spread (the
    group is then late in the whole problem too)."""
    its = _its()
    big, small = its
    t2 = {"matchExpressions": [{"key": synth.ZONE, "operator": "In", "values": ["test-zone-1"]}]}
    t1 = {"matchExpressions": [{"key": synth.ZONE, "operator": "In", "values": ["nowhere"]}]}
    spread = [{"maxSkew": 1, "topologyKey": synth.HOSTNAME, "whenUnsatisfiable": "DoNotSchedule",
               "labelSelector": {"matchLabels": {"app": "w"}}}]
    A = synth.pod(1, cpu="1", labels={"app": "w"},
                  affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [t2]}}},
                  extra={"topologySpreadConstraints": spread} if variant == 0 else None)
    B = synth.pod(2, cpu="1", labels={"app": "w"},
                  affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [t1, t2]}}},
                  extra={"topologySpreadConstraints": spread})
    B["spec"]["priority"] = 1
    cands = [mcf.node("cand-a", big, {"cpu": "1", "pods": "20"}, [_bound(A, "cand-a")]),
             mcf.node("cand-b", big, {"cpu": "1", "pods": "20"}, [_bound(B, "cand-b")])]
    keep = [mcf.node("keep-%d" % k, small, {"cpu": "4", "pods": "20"},
                     [_bound(synth.pod(10 + k, cpu="1", labels={"app": "q"}), "keep-%d" % k)]) for k in range(2)]
    w = mcf.node("keep-w", small, {"cpu": "4", "pods": "20"}, [_bound(synth.pod(20, cpu="3", labels={"app": "w"}), "keep-w")])
    nodes = cands + keep + [w]
    snap = mcf.snapshot(its, nodes)
    snap["candidates"] = ["cand-a", "cand-b"]
    snap["clusterPods"] = [copy.deepcopy(p) for n in nodes for p in n["pods"]]
    return snap
