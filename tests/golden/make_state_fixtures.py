#!/usr/bin/env python3
"""Known-answer cluster-state accounting scenarios hand-transcribed from the reference's Go tests.

Source: pkg/controllers/state/suite_test.go ("Node Resource Level", "Volume/HostPort usage",
"should not leak a state node ..."), with test.Node / test.Pod / test.NodeClaimAndNode defaults.
Each scenario is {"name", "source", "cluster", "expect"}: `cluster` is the converged object listing
({"nodeClaims", "nodes", "pods"}) after the test's events; `expect` holds the test's assertions:
  count       : number of StateNodes (ExpectStateNodeCount)
  nodes       : {node name: {"podRequests" / "daemonSetRequests": ResourceList (ExpectResources:
                every listed resource compares equal; missing = 0), "hostPorts": [ports reserved]}}
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
T0 = "2024-01-01T00:00:00Z"


def node(name, allocatable, labels=None, provider_id=None, taints=None, ready=True, capacity=None, deleting=False):
    md = {"name": name, "labels": dict(labels or {}), "creationTimestamp": T0}
    if deleting:
        md["deletionTimestamp"] = T0
    return {"metadata": md,
            "spec": {"providerID": provider_id if provider_id is not None else "fake:///" + name,
                     "taints": list(taints or [])},
            "status": {"allocatable": dict(allocatable), "capacity": dict(capacity or allocatable),
                       "conditions": [{"type": "Ready", "status": "True" if ready else "False"}]}}


def nodeclaim(name, provider_id, labels=None, allocatable=None, capacity=None, taints=None, startup_taints=None,
              deleting=False):
    md = {"name": name, "labels": dict(labels or {}), "creationTimestamp": T0}
    if deleting:
        md["deletionTimestamp"] = T0
    return {"metadata": md, "spec": {"taints": list(taints or []), "startupTaints": list(startup_taints or [])},
            "status": {"providerID": provider_id, "allocatable": dict(allocatable or {}),
                       "capacity": dict(capacity or allocatable or {})}}


def pod(name, requests=None, node_name="", phase="Running", daemonset=False, host_ports=(), ns="default", pvcs=()):
    c = {"name": "c", "resources": {"requests": dict(requests or {})}}
    if host_ports:
        c["ports"] = [{"containerPort": 8080, "hostPort": p, "protocol": "TCP"} for p in host_ports]
    md = {"name": name, "namespace": ns, "uid": "uid-" + ns + "-" + name, "creationTimestamp": T0}
    if daemonset:
        md["ownerReferences"] = [{"apiVersion": "apps/v1", "kind": "DaemonSet", "name": "ds", "uid": "ds-uid",
                                  "controller": True}]
    spec = {"nodeName": node_name, "containers": [c]}
    if pvcs:
        spec["volumes"] = [{"name": "v%d" % i, "persistentVolumeClaim": {"claimName": n}} for i, n in enumerate(pvcs)]
    return {"metadata": md, "spec": spec, "status": {"phase": phase}}


MANAGED = {"karpenter.sh/nodepool": "default", "node.kubernetes.io/instance-type": "1-cpu-1-mem-amd64-linux"}


def scenarios():
    src = "pkg/controllers/state/suite_test.go"
    S = []
    n = node("node-1", {"cpu": "4"}, MANAGED)
    p1, p2 = {"cpu": "1.5"}, {"cpu": "2"}
    S.append({"name": "pods-not-bound", "source": src + ":351-383",
              "cluster": {"nodes": [n], "pods": [pod("p1", p1), pod("p2", p2)]},
              "expect": {"count": 1, "nodes": {"node-1": {"podRequests": {"cpu": "0"}}}}})
    S.append({"name": "new-pods-bound", "source": src + ":384-423",
              "cluster": {"nodes": [n], "pods": [pod("p1", p1, "node-1"), pod("p2", p2, "node-1")]},
              "expect": {"count": 1, "nodes": {"node-1": {"podRequests": {"cpu": "3.5"}}}}})
    S.append({"name": "existing-pods-bound", "source": src + ":424-457",
              "cluster": {"nodes": [n], "pods": [pod("p1", p1, "node-1"), pod("p2", p2, "node-1")]},
              "expect": {"count": 1, "nodes": {"node-1": {"podRequests": {"cpu": "3.5"}}}}})
    S.append({"name": "pod-deleted", "source": src + ":458-503",
              "cluster": {"nodes": [n], "pods": [pod("p1", p1, "node-1")]},
              "expect": {"count": 1, "nodes": {"node-1": {"podRequests": {"cpu": "1.5"}}}}})
    S.append({"name": "all-pods-deleted", "source": src + ":458-503",
              "cluster": {"nodes": [n], "pods": []},
              "expect": {"count": 1, "nodes": {"node-1": {"podRequests": {"cpu": "0"}}}}})
    S.append({"name": "terminal-pods", "source": src + ":504-542",
              "cluster": {"nodes": [n], "pods": [pod("p1", p1, "node-1", phase="Failed"),
                                                 pod("p2", p2, "node-1", phase="Succeeded")]},
              "expect": {"count": 1, "nodes": {"node-1": {"podRequests": {"cpu": "0"}}}}})
    n2 = node("node-1", {"cpu": "4", "memory": "8Gi"}, MANAGED)
    S.append({"name": "daemonset-pod-not-bound", "source": src + ":726-775",
              "cluster": {"nodes": [n2], "pods": [pod("p1", p1, "node-1"),
                                                  pod("ds-pod", {"cpu": "1", "memory": "2Gi"}, daemonset=True)]},
              "expect": {"count": 1, "nodes": {"node-1": {"daemonSetRequests": {"cpu": "0", "memory": "0"},
                                                          "podRequests": {"cpu": "1.5"}}}}})
    S.append({"name": "daemonset-requests-separate", "source": src + ":726-802",
              "cluster": {"nodes": [n2], "pods": [pod("p1", p1, "node-1"),
                                                  pod("ds-pod", {"cpu": "1", "memory": "2Gi"}, "node-1",
                                                      daemonset=True)]},
              "expect": {"count": 1, "nodes": {"node-1": {"daemonSetRequests": {"cpu": "1", "memory": "2Gi"},
                                                          "podRequests": {"cpu": "2.5", "memory": "2Gi"}}}}})
    S.append({"name": "hostport-hydration", "source": src + ":235-257",
              "cluster": {"nodes": [node("node-1", {"cpu": "4"}, MANAGED)],
                          "pods": [pod("hp-%d" % i, None, "node-1", host_ports=[i]) for i in range(1, 10)]},
              "expect": {"count": 1, "nodes": {"node-1": {"hostPorts": [5]}}}})
    # "should hydrate the volume usage on a Node update" (:143-163): 10 bound pods with one PVC each of
    # a StorageClass provisioned by the CSI driver; the CSINode allows 10 volumes of that driver
    csi = "fake.csi.provider"
    S.append({"name": "volume-hydration", "source": src + ":100-163",
              "cluster": {"nodes": [node("node-1", {"cpu": "4"}, MANAGED)],
                          "pods": [pod("vp-%d" % i, None, "node-1", pvcs=["pvc-%d" % i]) for i in range(10)],
                          "volumeDrivers": {"default/pvc-%d" % i: csi for i in range(10)},
                          "csiNodes": [{"metadata": {"name": "node-1"},
                                        "spec": {"drivers": [{"name": csi, "allocatable": {"count": 10}}]}}]},
              "expect": {"count": 1, "nodes": {"node-1": {"volumes": {csi: 10}, "volumeLimits": {csi: 10}}}}})
    nc = nodeclaim("nodeclaim-1", "fake:///nodeclaim-1", MANAGED, {"cpu": "4"})
    S.append({"name": "nodeclaim-and-node-same-name", "source": src + ":323-350",
              "cluster": {"nodeClaims": [nc], "nodes": [node("nodeclaim-1", {"cpu": "4"}, MANAGED)], "pods": []},
              "expect": {"count": 1, "nodes": {}}})
    S.append({"name": "nodeclaim-deleted-node-remains", "source": src + ":341-346",
              "cluster": {"nodeClaims": [], "nodes": [node("nodeclaim-1", {"cpu": "4"}, MANAGED)], "pods": []},
              "expect": {"count": 1, "nodes": {}}})
    S.append({"name": "both-deleted", "source": src + ":347-349",
              "cluster": {"nodeClaims": [], "nodes": [], "pods": []}, "expect": {"count": 0, "nodes": {}}})
    return S


def main():
    out = [{"name": s["name"], "source": s["source"], "expect": s["expect"]} for s in scenarios()]
    with open(os.path.join(HERE, "state_scenarios.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("%d state scenarios" % len(out))


if __name__ == "__main__":
    main()
