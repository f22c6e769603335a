#!/usr/bin/env python3
"""Known-answer consolidation scenarios hand-transcribed from the reference's Go tests.

Source: pkg/controllers/disruption/consolidation_test.go, with the suite setup of
pkg/controllers/disruption/suite_test.go:95-130 (fake.InstanceTypesAssorted(), on-demand types
sorted by cheapest price -> leastExpensiveInstance / mostExpensiveInstance) and the test.NodePool()
defaults (WhenUnderutilized, expireAfter 720h; clock stepped 10 minutes past node creation).

Each scenario is {"name", "source", "snapshot", "expect"}; `expect` holds the Go test's assertion on
the command the disruption controller would execute (multi-node consolidation runs before
single-node consolidation; the first non-no-op wins):
  action      : "delete" | "replace" | "no-op"
  candidates  : node names removed by the command (set)
  replacement_excludes : an instance type the replacement must not offer

validation_scenarios() transcribes the TTL-wait tests (consolidation_test.go:2212-2562): a command is
computed on the snapshot `before`, the cluster changes during Validation's wait, and
Validation.IsValid (validation.go:68-180) re-checks it against `after`.  `expect.valid` is the Go
test's outcome (the node is kept when the command is invalid); `expect.reason` names the check.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "karpenter-sigs_amd"))
from karpenter_amd import synth  # noqa: E402

NOW = synth.NOW


def assorted():
    """fake.InstanceTypesAssorted (fake/instancetype.go:111-145)."""
    out = []
    for cpu in [1, 2, 4, 8, 16, 32, 64]:
        for mem in [1, 2, 4, 8, 16, 32, 64, 128]:
            for zone in ["test-zone-1", "test-zone-2", "test-zone-3"]:
                for ct in ["spot", "on-demand"]:
                    for os_ in ["linux", "windows"]:
                        for arch in ["amd64", "arm64"]:
                            name = "%d-cpu-%d-mem-%s-%s-%s-%s" % (cpu, mem, arch, os_, zone, ct)
                            price = synth.price_from_resources(cpu, mem * synth.GI)
                            out.append(synth.fake_instance_type(
                                name, cpu, mem, pods=None, arch=arch, oses=(os_,),
                                offerings=[{"capacityType": ct, "zone": zone, "price": price, "available": True}]))
    return out


def cheapest_price(it):
    return min(o["price"] for o in it["offerings"])


def od_sorted(its):
    # suite_test.go:116-128; price ties keep list order here (Go's sort.Slice tie order is unpinned,
    # and no assertion below depends on which tied type is picked)
    ods = [it for it in its if any(o["capacityType"] == "on-demand" for o in it["offerings"])]
    return sorted(ods, key=cheapest_price)


def nodepool(requirements=None, disruption=None):
    np_ = synth.node_pool("default", requirements=requirements)
    np_["spec"]["disruption"] = {"consolidationPolicy": "WhenUnderutilized", "expireAfter": "720h"}
    np_["spec"]["disruption"].update(disruption or {})
    return np_


def rs_pod(i, cpu=None, bound_to=None, annotations=None, pending=False):
    """test.Pod owned by a ReplicaSet (consolidation_test.go), bound with ExpectManualBinding."""
    p = synth.pod(i, cpu=cpu)
    p["metadata"]["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "ReplicaSet", "name": "rs", "uid": "rs-uid"}]
    p["metadata"]["labels"] = {"app": "test"}
    if annotations:
        p["metadata"]["annotations"] = annotations
    if bound_to:
        p["spec"]["nodeName"] = bound_to
        p["status"] = {"phase": "Running", "conditions": [{"type": "PodScheduled", "status": "True"}]}
    return p


def node(name, it, alloc, pods, initialized=True, annotations=None):
    """test.NodeClaimAndNode with the NodeClaim's labels, annotations and Status.Allocatable."""
    off = it["offerings"][0]
    labels = {synth.NODEPOOL: "default", synth.IT_LABEL: it["name"], synth.CT: off["capacityType"],
              synth.ZONE: off["zone"], synth.HOSTNAME: name}
    avail = dict(alloc)
    if "pods" in avail:
        avail["pods"] = str(int(avail["pods"]) - len(pods))
    if "cpu" in avail:
        used_m = 0
        for p in pods:
            c = p["spec"]["containers"][0]["resources"]["requests"].get("cpu")
            if c:
                used_m += int(float(c) * 1000) if not c.endswith("m") else int(c[:-1])
        total_m = int(float(alloc["cpu"]) * 1000)
        avail["cpu"] = "%dm" % (total_m - used_m)
    out = {"name": name, "hostName": name, "labels": labels, "taints": [], "capacity": dict(alloc),
           "available": avail, "daemonSetRequests": {}, "initialized": initialized, "ready": initialized,
           "creationTimestamp": synth._fmt_time(NOW - 600), "pods": pods}
    if annotations:  # NodeClaimLinkedNode copies the NodeClaim's annotations (pkg/test/nodes.go:70-84)
        out["annotations"] = dict(annotations)
    return out


def snapshot(its, nodes, pending=(), requirements=None, disruption=None):
    np_ = nodepool(requirements, disruption)
    return {"wellKnownLabels": synth.FAKE_WELL_KNOWN, "instanceTypes": its,
            "instanceTypesByNodePool": {"default": list(range(len(its)))},
            "nodeClaimTemplates": [np_], "nodePools": [np_], "daemonSetPods": [],
            "stateNodes": nodes, "pendingPods": list(pending), "candidates": [n["name"] for n in nodes],
            "now": synth._fmt_time(NOW), "hostnameSeed": 0}


def scenarios():
    src = "pkg/controllers/disruption/consolidation_test.go"
    its = assorted()
    ods = od_sorted(its)
    least, most = ods[0], ods[-1]
    S = []
    # Replace / "can replace node" (:209-266)
    n = node("node-a", most, {"cpu": "32"}, [rs_pod(0, bound_to="node-a")])
    S.append({"name": "can-replace-node", "source": src + ":209-266", "snapshot": snapshot(its, [n]),
              "expect": {"action": "replace", "candidates": ["node-a"], "replacement_excludes": most["name"]}})
    # "won't replace node if any spot replacement is more expensive" (:851-945)
    cur = synth.fake_instance_type("current-on-demand", 4, 4, offerings=[
        {"capacityType": "on-demand", "zone": "test-zone-1a", "price": 0.5, "available": False}])
    rep = synth.fake_instance_type("potential-spot-replacement", 4, 4, offerings=[
        {"capacityType": "spot", "zone": "test-zone-1a", "price": 1.0, "available": True},
        {"capacityType": "spot", "zone": "test-zone-1b", "price": 0.2, "available": True},
        {"capacityType": "spot", "zone": "test-zone-1c", "price": 0.4, "available": True}])
    n = node("node-a", cur, {"cpu": "32"}, [rs_pod(0, bound_to="node-a")])
    S.append({"name": "spot-replacement-more-expensive", "source": src + ":851-945",
              "snapshot": snapshot([cur, rep], [n]), "expect": {"action": "no-op", "candidates": []}})
    # "won't replace on-demand node if on-demand replacement is more expensive" (:946-1040)
    rep = synth.fake_instance_type("on-demand-replacement", 4, 4, offerings=[
        {"capacityType": "on-demand", "zone": "test-zone-1a", "price": 0.6, "available": True},
        {"capacityType": "on-demand", "zone": "test-zone-1b", "price": 0.6, "available": True},
        {"capacityType": "spot", "zone": "test-zone-1b", "price": 0.2, "available": True},
        {"capacityType": "spot", "zone": "test-zone-1c", "price": 0.3, "available": True}])
    n = node("node-a", cur, {"cpu": "32"}, [rs_pod(0, bound_to="node-a")])
    S.append({"name": "on-demand-replacement-more-expensive", "source": src + ":946-1040",
              "snapshot": snapshot([cur, rep], [n], requirements=[
                  {"key": synth.CT, "operator": "In", "values": ["on-demand"]}]),
              "expect": {"action": "no-op", "candidates": []}})
    # Delete / "can delete nodes" (:1098-1145)
    alloc = {"cpu": "32", "pods": "100"}
    n1 = node("node-a", least, alloc, [rs_pod(0, bound_to="node-a"), rs_pod(1, bound_to="node-a")])
    n2 = node("node-b", least, alloc, [rs_pod(2, bound_to="node-b")])
    S.append({"name": "can-delete-nodes", "source": src + ":1098-1145", "snapshot": snapshot(its, [n1, n2]),
              "expect": {"action": "delete", "candidates": ["node-b"]}})
    # "won't delete node if it would require pods to schedule on an un-initialized node" (:1582-1631)
    n1 = node("node-a", least, alloc, [rs_pod(0, bound_to="node-a"), rs_pod(1, bound_to="node-a")],
              initialized=False)
    n2 = node("node-b", least, alloc, [rs_pod(2, bound_to="node-b")])
    S.append({"name": "no-delete-onto-uninitialized", "source": src + ":1582-1631",
              "snapshot": snapshot(its, [n1, n2]), "expect": {"action": "no-op", "candidates": []}})
    # "can replace nodes, considers karpenter.sh/do-not-disrupt on pods" (:772-850)
    n = node("node-a", most, {"cpu": "32"},
             [rs_pod(0, bound_to="node-a", annotations={"karpenter.sh/do-not-disrupt": "true"})])
    S.append({"name": "do-not-disrupt-pod", "source": src + ":772-850", "snapshot": snapshot(its, [n]),
              "expect": {"action": "no-op", "candidates": []}})
    # "considers pending pods when consolidating" (:148-208)
    large = sorted([it for it in its if int(it["capacity"]["cpu"]) >= 64], key=lambda it: it["offerings"][0]["price"])[0]
    bound = rs_pod(0, cpu="1", bound_to="node-a")
    bound["metadata"].pop("ownerReferences")
    unsched = synth.pod(1, cpu="62")
    n = node("node-a", large, {"cpu": large["capacity"]["cpu"], "pods": large["capacity"]["pods"]}, [bound])
    S.append({"name": "considers-pending-pods", "source": src + ":148-208",
              "snapshot": snapshot(its, [n], pending=[unsched]), "expect": {"action": "no-op", "candidates": []}})
    # Multi-NodeClaim / "can merge 3 nodes into 1" (:2799-2848)
    ns = [node("node-%s" % c, most, alloc, [rs_pod(i, bound_to="node-%s" % c)]) for i, c in enumerate("abc")]
    S.append({"name": "merge-3-into-1", "source": src + ":2799-2848", "snapshot": snapshot(its, ns),
              "expect": {"action": "replace", "candidates": ["node-a", "node-b", "node-c"]}})
    # "won't merge 2 nodes into 1 of the same type" (:2849-2926)
    n1 = node("node-a", least, alloc, [rs_pod(0, bound_to="node-a")])
    n2 = node("node-b", least, alloc, [rs_pod(1, bound_to="node-b"), rs_pod(2, bound_to="node-b")])
    S.append({"name": "no-merge-same-type", "source": src + ":2849-2926", "snapshot": snapshot(its, [n1, n2]),
              "expect": {"action": "delete", "candidates": ["node-a"]}})
    # Node annotations block candidates: NewCandidate's do-not-disrupt key (types.go:78-81) and
    # ShouldDisrupt's do-not-consolidate == "true" (consolidation.go:96-101).
    # "can delete nodes, considers karpneter.sh/do-not-consolidate on nodes" (:1319-1370) and
    # "... karpenter.sh/do-not-disrupt on nodes" (:1371-1422): the non-annotated node (more pods) goes
    for key, lines in (("karpenter.sh/do-not-consolidate", "1319-1370"), ("karpenter.sh/do-not-disrupt", "1371-1422")):
        n1 = node("node-a", least, alloc, [rs_pod(0, bound_to="node-a"), rs_pod(1, bound_to="node-a")])
        n2 = node("node-b", least, alloc, [rs_pod(2, bound_to="node-b")], annotations={key: "true"})
        S.append({"name": "delete-considers-%s-on-nodes" % key.split("/")[1], "source": src + ":" + lines,
                  "snapshot": snapshot(its, [n1, n2]), "expect": {"action": "delete", "candidates": ["node-a"]}})
    # "can replace nodes, considers karpenter.sh/do-not-consolidate on nodes" (:536-614) and
    # "... karpenter.sh/do-not-disrupt on nodes" (:615-693): 2 pods of 2 cpu on the 32-cpu node are
    # replaced; the annotated 5-cpu node keeps its pod
    for key, lines in (("karpenter.sh/do-not-consolidate", "536-614"), ("karpenter.sh/do-not-disrupt", "615-693")):
        n1 = node("node-a", most, {"cpu": "32"}, [rs_pod(0, cpu="2", bound_to="node-a"), rs_pod(1, cpu="2", bound_to="node-a")])
        n2 = node("node-b", most, {"cpu": "5", "pods": "100"}, [rs_pod(2, cpu="2", bound_to="node-b")],
                  annotations={key: "true"})
        S.append({"name": "replace-considers-%s-on-nodes" % key.split("/")[1], "source": src + ":" + lines,
                  "snapshot": snapshot(its, [n1, n2]),
                  "expect": {"action": "replace", "candidates": ["node-a"], "replacement_excludes": most["name"]}})
    # ShouldDisrupt's NodePool rule (consolidation.go:102-106): consolidation is disabled for a pool whose
    # consolidationPolicy is not WhenUnderutilized, or whose consolidateAfter is Never
    for tag, dis in (("when-empty-policy", {"consolidationPolicy": "WhenEmpty", "consolidateAfter": "30s"}),
                     ("consolidate-after-never", {"consolidateAfter": "Never"})):
        n1 = node("node-a", least, alloc, [rs_pod(0, bound_to="node-a"), rs_pod(1, bound_to="node-a")])
        n2 = node("node-b", least, alloc, [rs_pod(2, bound_to="node-b")])
        S.append({"name": "pool-%s-disables-consolidation" % tag,
                  "source": "pkg/controllers/disruption/consolidation.go:102-106",
                  "snapshot": snapshot(its, [n1, n2], disruption=dis), "expect": {"action": "no-op", "candidates": []}})
    # A node nominated for a pending pod is not a candidate (NewCandidate, types.go:110-113)
    n1 = node("node-a", least, alloc, [rs_pod(0, bound_to="node-a"), rs_pod(1, bound_to="node-a")])
    n2 = node("node-b", least, alloc, [rs_pod(2, bound_to="node-b")])
    n2["nominated"] = True
    S.append({"name": "nominated-node-is-not-a-candidate", "source": "pkg/controllers/disruption/types.go:110-113",
              "snapshot": snapshot(its, [n1, n2]), "expect": {"action": "delete", "candidates": ["node-a"]}})
    return S


def blocking_pdb(app):
    """test.PodDisruptionBudget(MaxUnavailable 0) over app=<app>: no disruptions allowed."""
    return {"metadata": {"name": "pdb-" + app, "namespace": "default"},
            "spec": {"selector": {"matchLabels": {"app": app}}}, "status": {"disruptionsAllowed": 0}}


def validation_scenarios():
    src = "pkg/controllers/disruption/consolidation_test.go"
    its = assorted()
    ods = od_sorted(its)
    least, most = ods[0], ods[-1]
    alloc = {"cpu": "32", "pods": "100"}
    dnd = {"karpenter.sh/do-not-disrupt": "true"}
    V = []

    def blocker(i, bound_to, app="blocking"):
        p = rs_pod(i, bound_to=bound_to)
        p["metadata"]["labels"] = {"app": app}
        return p

    # "should not consolidate if the action becomes invalid during the node TTL wait" (:2212-2250):
    # an empty node is deleted, then a do-not-disrupt pod binds to it
    before = snapshot(its, [node("node-a", least, alloc, [])])
    after = snapshot(its, [node("node-a", least, alloc, [rs_pod(0, bound_to="node-a", annotations=dnd)])])
    V.append({"name": "empty-node-gets-do-not-disrupt-pod", "source": src + ":2212-2250", "before": before,
              "after": after, "expect": {"command": "delete", "valid": False, "reason": "candidates-changed"}})
    # "should not replace node if a pod schedules with a blocking PDB during the TTL wait" (:2351-2404)
    before = snapshot(its, [node("node-a", most, {"cpu": "32"}, [rs_pod(0, bound_to="node-a")])])
    after = snapshot(its, [node("node-a", most, {"cpu": "32"}, [rs_pod(0, bound_to="node-a"),
                                                                blocker(1, "node-a")])])
    after["podDisruptionBudgets"] = [blocking_pdb("blocking")]
    V.append({"name": "replace-blocked-by-pdb-during-wait", "source": src + ":2351-2404", "before": before,
              "after": after, "expect": {"command": "replace", "valid": False, "reason": "candidates-changed"}})
    # "should not delete node if pods schedule with karpenter.sh/do-not-disrupt during the TTL wait"
    # (:2455-2505) and "... with a blocking PDB during the TTL wait" (:2506-2562): two nodes, one deleted
    two = lambda extra: [node("node-a", least, alloc, [rs_pod(0, bound_to="node-a")] + extra[0]),
                         node("node-b", least, alloc, [rs_pod(1, bound_to="node-b")] + extra[1])]
    before = snapshot(its, two(([], [])))
    after = snapshot(its, two(([rs_pod(2, bound_to="node-a", annotations=dnd)],
                               [rs_pod(3, bound_to="node-b", annotations=dnd)])))
    V.append({"name": "delete-blocked-by-do-not-disrupt-during-wait", "source": src + ":2455-2505",
              "before": before, "after": after,
              "expect": {"command": "delete", "valid": False, "reason": "candidates-changed"}})
    after = snapshot(its, two(([blocker(2, "node-a")], [blocker(3, "node-b")])))
    after["podDisruptionBudgets"] = [blocking_pdb("blocking")]
    V.append({"name": "delete-blocked-by-pdb-during-wait", "source": src + ":2506-2562",
              "before": before, "after": after,
              "expect": {"command": "delete", "valid": False, "reason": "candidates-changed"}})
    # Unchanged clusters: every consolidation test above passes Validation (ValidateCommand :135-180)
    for sc in scenarios():
        if sc["name"] in ("can-replace-node", "can-delete-nodes", "merge-3-into-1", "no-merge-same-type"):
            V.append({"name": "unchanged-" + sc["name"], "source": "pkg/controllers/disruption/validation.go:120-180",
                      "before": sc["snapshot"], "after": sc["snapshot"],
                      "expect": {"command": sc["expect"]["action"], "valid": True, "reason": ""}})
    # A pending pod nominated to the candidate during the wait: NewCandidate drops a nominated node
    # (types.go:110-113), so the candidate no longer maps and the command is invalid before the
    # IsNodeNominated check of validation.go:99-103 is reached
    before = snapshot(its, two(([], [])))
    after = snapshot(its, two(([], [])))
    for n in after["stateNodes"]:
        n["nominated"] = True
    V.append({"name": "candidate-nominated-during-wait", "source": "pkg/controllers/disruption/types.go:110-113",
              "before": before, "after": after,
              "expect": {"command": "delete", "valid": False, "reason": "candidates-changed"}})
    # The pool's consolidateAfter turns to Never during the wait: Validation.ShouldDisrupt checks only the
    # policy and do-not-consolidate (validation.go:112-118), so the command is still valid
    after = snapshot(its, two(([], [])), disruption={"consolidateAfter": "Never"})
    V.append({"name": "consolidate-after-never-during-wait", "source": "pkg/controllers/disruption/validation.go:112-118",
              "before": before, "after": after, "expect": {"command": "delete", "valid": True, "reason": ""}})
    # ... while a do-not-consolidate annotation added during the wait invalidates it
    after = snapshot(its, two(([], [])))
    for n in after["stateNodes"]:
        n["annotations"] = {"karpenter.sh/do-not-consolidate": "true"}
    V.append({"name": "do-not-consolidate-during-wait", "source": "pkg/controllers/disruption/validation.go:112-118",
              "before": before, "after": after,
              "expect": {"command": "delete", "valid": False, "reason": "candidates-changed"}})
    # The deleted node's pods no longer fit elsewhere: re-simulation wants a NodeClaim (validation.go:155-160)
    after = snapshot(its, two(([], [])))
    for n in after["stateNodes"]:  # whichever node is deleted, the other one is now full
        n["available"]["pods"] = "0"
    V.append({"name": "deleted-pods-need-a-new-node", "source": "pkg/controllers/disruption/validation.go:155-160",
              "before": before, "after": after,
              "expect": {"command": "delete", "valid": False, "reason": "replacement-needed"}})
    return V


def main():
    # The snapshots (1344 instance types each) are rebuilt from this script by the tests; the fixture
    # keeps the transcribed expectations.
    out = [{"name": s["name"], "source": s["source"], "expect": s["expect"]} for s in scenarios()]
    with open(os.path.join(HERE, "consolidation_scenarios.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("%d scenarios" % len(out))
    out = [{"name": s["name"], "source": s["source"], "expect": s["expect"]} for s in validation_scenarios()]
    with open(os.path.join(HERE, "validation_scenarios.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("%d validation scenarios" % len(out))


if __name__ == "__main__":
    main()
