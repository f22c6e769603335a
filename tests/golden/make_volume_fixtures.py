#!/usr/bin/env python3
"""Known-answer volume-limit scenarios hand-transcribed from the reference's Go tests.

Source: pkg/controllers/provisioning/scheduling/suite_test.go, Describe("VolumeUsage") (:2656-3420).
Every scenario first provisions an initial pod (ExpectProvisioned), registers a CSINode with per-driver
allocatable counts for the node it landed on, then provisions more pods.  The snapshot starts at the
second ExpectProvisioned: the node is an existing, initialized StateNode carrying the initial pod's
volume usage and the CSINode limits (cluster.go:468 -> VolumeUsage.AddLimit).  PVC -> CSI driver
resolution (resolveDriver, volumeusage.go:115-172: PV CSI driver, in-tree translation, storage-class
provisioner, the apiserver's default storage class) happens while the snapshot is built, so it is an
input here ("volumeDrivers"); an empty driver (NFS PV, no storage class) is skipped by GetVolumes.

`expect`: new_claims = NewNodeClaims created by the second Solve (the Go tests assert the node count,
i.e. 1 + new_claims); existing_pods = how many pods land on the existing node; scheduled = True.
Run with --write to regenerate volume_scenarios.json.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "karpenter-sigs_amd"))
from karpenter_amd import synth  # noqa: E402

SRC = "pkg/controllers/provisioning/scheduling/suite_test.go:"
CSI = "fake.csi.provider"  # suite_test.go:74
EBS = "ebs.csi.aws.com"    # plugins.AWSEBSDriverName (csi-translation-lib)


def instance_types():
    # VolumeUsage BeforeEach (:2657-2669): one type, 1024 cpu / 1024 pods (memory defaults to 4Gi)
    return [synth.fake_instance_type("instance-type", 1024, 4, pods=1024)]


def existing_node(usage, limits):
    """The node the initial pod landed on: Available = Allocatable - the initial pod (pods=1)."""
    return {
        "name": "node-initial", "hostName": "node-initial",
        "labels": {synth.NODEPOOL: "default", synth.IT_LABEL: "instance-type", synth.ZONE: "test-zone-1",
                   synth.CT: "spot", synth.ARCH: "amd64", synth.OS: "linux", synth.HOSTNAME: "node-initial"},
        "taints": [],
        "available": {"cpu": "1023900m", "memory": "4086Mi", "pods": "1023"},
        "capacity": {"cpu": "1024", "memory": "4Gi", "pods": "1024"},
        "initialized": True,
        "volumeUsage": usage,
        "volumeLimits": limits,
    }


def pvc_pod(i, claims=(), ephemeral=()):
    vols = [{"name": "v%d" % k, "persistentVolumeClaim": {"claimName": c}} for k, c in enumerate(claims)]
    vols += [{"name": v, "ephemeral": {"volumeClaimTemplate": {"spec": {}}}} for v in ephemeral]
    p = synth.pod(i, extra={"volumes": vols} if vols else None)
    return p


def snapshot(pods, node, drivers):
    its = instance_types()
    pool = synth.node_pool("default", requirements=[{"key": synth.CT, "operator": "In",
                                                      "values": ["spot", "on-demand"]}])
    return {
        "wellKnownLabels": synth.FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": {"default": [0]},
        "nodeClaimTemplates": [pool],
        "nodePools": [pool],
        "stateNodes": [node],
        "daemonSetPods": [],
        "pods": pods,
        "volumeDrivers": drivers,
    }


def scenarios():
    out = []

    def add(name, line, pods, node, drivers, expect):
        out.append({"name": name, "source": SRC + line, "snapshot": snapshot(pods, node, drivers), "expect": expect})

    # 6 pods x 2 unbound PVCs of my-storage-class (provisioner fake.csi.provider), node limit 10:
    # five pods fit the existing node, the sixth needs a new node (:2670-2720)
    pods = [pvc_pod(i, ["my-claim-a-%d" % i, "my-claim-b-%d" % i]) for i in range(6)]
    drivers = {"default/my-claim-%s-%d" % (ab, i): CSI for i in range(6) for ab in "ab"}
    add("volume-limits-multiple-nodes", "2670-2720", pods, existing_node({}, {CSI: 10}), drivers,
        {"new_claims": 1, "existing_pods": 5, "scheduled": True})
    # 100 pods sharing one PVC bound to a CSI PV (test.PersistentVolume: driver test.driver) (:2721-2772)
    pods = [pvc_pod(i, ["my-claim"]) for i in range(100)]
    add("same-pvc-single-node", "2721-2772", pods, existing_node({}, {CSI: 10}),
        {"default/my-claim": "test.driver"}, {"new_claims": 0, "existing_pods": 100, "scheduled": True})
    # NFS PV (no CSI source) with storageClassName "": resolveDriver returns "" and the PVC is skipped (:2773-2805)
    pods = [pvc_pod(i, ["my-claim", "my-claim"]) for i in range(5)]
    add("nfs-volumes", "2773-2805", pods, existing_node({}, {}), {"default/my-claim": ""},
        {"new_claims": 0, "existing_pods": 5, "scheduled": True})
    # ephemeral volume with my-storage-class; the node holds the initial pod's ephemeral PVC, limit 1 (:2806-2880)
    init_pvc = "default/pod-initial-tmp-ephemeral"
    p = pvc_pod(0, ephemeral=["tmp-ephemeral"])
    add("ephemeral-specified-storage-class", "2806-2880", [p],
        existing_node({CSI: [init_pvc]}, {CSI: 1, "other-provider": 10}),
        {"default/pod-000000-tmp-ephemeral": CSI}, {"new_claims": 1, "existing_pods": 0, "scheduled": True})
    # ephemeral volume without a storage class: the apiserver defaults the PVC to the default class (:2881-2960)
    p = pvc_pod(0, ephemeral=["tmp-ephemeral"])
    add("ephemeral-default-storage-class", "2881-2960", [p], existing_node({CSI: [init_pvc]}, {CSI: 1}),
        {"default/pod-000000-tmp-ephemeral": CSI}, {"new_claims": 1, "existing_pods": 0, "scheduled": True})
    # two default classes: the newest (provisioner fake.csi.provider) wins (:3020-3100)
    p = pvc_pod(0, ephemeral=["tmp-ephemeral"])
    add("ephemeral-newest-storage-class", "3020-3100", [p],
        existing_node({CSI: [init_pvc]}, {CSI: 1, "other-provider": 10}),
        {"default/pod-000000-tmp-ephemeral": CSI}, {"new_claims": 1, "existing_pods": 0, "scheduled": True})
    # CSIMigration: in-tree kubernetes.io/aws-ebs storage class translates to ebs.csi.aws.com (:3228-3290)
    p = pvc_pod(0, ["pvc-2"])
    add("csi-migration-non-dynamic", "3228-3290", [p], existing_node({EBS: ["default/pvc-1"]}, {EBS: 1}),
        {"default/pvc-1": EBS, "default/pvc-2": EBS}, {"new_claims": 1, "existing_pods": 0, "scheduled": True})
    # CSIMigration, ephemeral volumes (:3291-3380)
    p = pvc_pod(0, ephemeral=["tmp-ephemeral"])
    add("csi-migration-ephemeral", "3291-3380", [p], existing_node({EBS: [init_pvc]}, {EBS: 1}),
        {"default/pod-000000-tmp-ephemeral": EBS}, {"new_claims": 1, "existing_pods": 0, "scheduled": True})
    return out


def check(scn, res):
    exp = scn["expect"]
    bad = []
    if len(res["newNodeClaims"]) != exp["new_claims"]:
        bad.append("%d new NodeClaims, want %d" % (len(res["newNodeClaims"]), exp["new_claims"]))
    on_existing = sum(len(n["pods"]) for n in res["existingNodes"])
    if on_existing != exp["existing_pods"]:
        bad.append("%d pods on the existing node, want %d" % (on_existing, exp["existing_pods"]))
    if exp["scheduled"] is True and res["podErrors"]:
        bad.append("unschedulable: %s" % sorted(res["podErrors"]))
    return bad


def main():
    fx = [{"name": s["name"], "source": s["source"], "expect": s["expect"]} for s in scenarios()]
    if "--write" in sys.argv:
        with open(os.path.join(HERE, "volume_scenarios.json"), "w") as f:
            json.dump(fx, f, indent=1)
    print(json.dumps(fx, indent=1))


if __name__ == "__main__":
    main()
