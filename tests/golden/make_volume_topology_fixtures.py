#!/usr/bin/env python3
"""Known-answer volume-topology scenarios hand-transcribed from the reference's Go tests.

Source: pkg/controllers/provisioning/suite_test.go, Context("Volume Topology Requirements") (:1155-1436).
Each test applies a NodePool and PVC / PV / StorageClass objects (pkg/test/storage.go builders), then calls
ExpectProvisioned, i.e. Provisioner.Schedule: GetPendingPods (which drops pods failing
ValidatePersistentVolumeClaims, provisioner.go:156-178,411-418), then NewScheduler (injectTopology, then
NewTopology, provisioner.go:204-296) and Solve.

The snapshot here is what NewScheduler receives: its "pods" are the pending pods that pass Validate's PVC
check (get_pending_pods below restates volumetopology.go:144-191 for the harness; Validate is GetPendingPods'
business, not the scheduler's).  The PVC / PV / StorageClass objects travel in the snapshot, and the
library runs VolumeTopology.Inject itself.

`expect` per pod name: "zone" (the NodeClaim the pod lands on is restricted to that zone -- the Go test
reads the launched node's zone label), True (scheduled) or False (not scheduled: dropped by GetPendingPods,
or a PodErrors entry).  Run with --write to regenerate volume_topology_scenarios.json.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "karpenter-sigs_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
from karpenter_amd import synth  # noqa: E402
import make_scenario_fixtures as msf  # noqa: E402

SRC = "pkg/controllers/provisioning/suite_test.go:"


def storage_class(name, zones=None, provisioner="test-provisioner"):
    """test.StorageClass (pkg/test/storage.go:117-141)."""
    sc = {"metadata": {"name": name}, "provisioner": provisioner}
    if zones is not None:
        sc["allowedTopologies"] = [{"matchLabelExpressions": [{"key": synth.ZONE, "values": zones}]}]
    return sc


def pv(name, zones=None, storage_class="", driver="test.driver"):
    """test.PersistentVolume (storage.go:39-85): a CSI source, zones as a required node affinity term."""
    spec = {"csi": {"driver": driver, "volumeHandle": "test-handle"}, "storageClassName": storage_class,
            "accessModes": ["ReadWriteOnce"], "capacity": {"storage": "100Gi"}}
    if zones:
        spec["nodeAffinity"] = {"required": {"nodeSelectorTerms": [
            {"matchExpressions": [{"key": synth.ZONE, "operator": "In", "values": zones}]}]}}
    return {"metadata": {"name": name}, "spec": spec}


def pvc(name, storage_class=None, volume_name="", namespace="default"):
    """test.PersistentVolumeClaim (storage.go:87-115): storageClassName is a pointer (None = nil)."""
    spec = {"accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}}}
    if storage_class is not None:
        spec["storageClassName"] = storage_class
    if volume_name:
        spec["volumeName"] = volume_name
    return {"metadata": {"name": name, "namespace": namespace}, "spec": spec}


def pod(i, claims=(), ephemeral=(), node_requirements=None, extra_terms=None):
    """test.UnschedulablePod with PersistentVolumeClaims / EphemeralVolumeTemplates / NodeRequirements
    (pkg/test/pods.go:72-110,221-290)."""
    vols = [{"name": "vol-%d" % k, "persistentVolumeClaim": {"claimName": c}} for k, c in enumerate(claims)]
    for k, sc in enumerate(ephemeral):
        vols.append({"name": "eph-%d" % k, "ephemeral": {"volumeClaimTemplate": {"spec": {
            "accessModes": ["ReadWriteOnce"], "resources": {"requests": {"storage": "1Gi"}},
            **({"storageClassName": sc} if sc is not None else {})}}}})
    extra = {"volumes": vols} if vols else {}
    affinity = None
    if node_requirements is not None:
        terms = [{"matchExpressions": node_requirements}] + list(extra_terms or [])
        affinity = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": terms}}}
    return synth.pod(i, affinity=affinity, extra=extra or None)


def ephemeral_claim(p, k=0):
    return "%s-%s" % (p["metadata"]["name"], p["spec"]["volumes"][k]["name"])


def get_pending_pods(pods, pvcs, pvs, scs):
    """GetPendingPods' Validate, PVC part (ValidatePersistentVolumeClaims, volumetopology.go:144-191): a pod
    whose claim is missing, whose bound volume is missing, or whose unbound claim names no storage class or a
    missing one is dropped (provisioner.go:169-172).  Harness only: the library starts at NewScheduler."""
    claims = {(c["metadata"]["namespace"], c["metadata"]["name"]): c for c in pvcs}
    vols = {v["metadata"]["name"] for v in pvs}
    classes = {s["metadata"]["name"] for s in scs}
    keep, dropped = [], []
    for p in pods:
        ok = True
        for v in p["spec"].get("volumes", []):
            if "persistentVolumeClaim" in v:
                name = v["persistentVolumeClaim"]["claimName"]
            elif "ephemeral" in v:
                name = "%s-%s" % (p["metadata"]["name"], v["name"])
            else:
                continue
            c = claims.get((p["metadata"]["namespace"], name))
            if c is None:
                ok = False
                break
            if c["spec"].get("volumeName"):
                ok = c["spec"]["volumeName"] in vols
            else:
                sc = c["spec"].get("storageClassName") or ""
                ok = sc != "" and sc in classes
            if not ok:
                break
        (keep if ok else dropped).append(p)
    return keep, dropped


def snapshot(pods, pvcs=(), pvs=(), scs=()):
    """The provisioning suite: fake.NewCloudProvider's default instance types, one test.NodePool() (no
    requirements, cpu limit 2000, pkg/test/nodepool.go:33-61)."""
    its = msf.default_instance_types()
    np_obj = synth.node_pool("default", limits={"cpu": "2000"})
    keep, dropped = get_pending_pods(pods, list(pvcs), list(pvs), list(scs))
    snap = {
        "wellKnownLabels": synth.FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": {"default": list(range(len(its)))},
        "nodeClaimTemplates": [np_obj],
        "nodePools": [np_obj],
        "stateNodes": [],
        "daemonSetPods": [],
        "pods": keep,
        "persistentVolumeClaims": list(pvcs),
        "persistentVolumes": list(pvs),
        "storageClasses": list(scs),
    }
    return snap, [p["metadata"]["name"] for p in dropped]


def scenarios():
    out = []
    SC = storage_class("my-storage-class", zones=["test-zone-2", "test-zone-3"])  # BeforeEach (:1157-1159)

    def add(name, lines, pods, expect, pvcs=(), pvs=(), scs=()):
        snap, dropped = snapshot(pods, pvcs, pvs, scs)
        out.append({"name": name, "source": SRC + lines, "snapshot": snap, "dropped": dropped,
                    "expect": {p["metadata"]["name"]: e for p, e in zip(pods, expect)}})

    add("invalid-pvc", "1160-1167", [pod(0, claims=["invalid"])], [False])
    add("empty-class-bound", "1168-1187", [pod(0, claims=["claim"])], [True],
        pvcs=[pvc("claim", storage_class="", volume_name="test-volume")], pvs=[pv("test-volume", storage_class="")])
    add("empty-class-unbound", "1188-1197", [pod(0, claims=["claim"])], [False], pvcs=[pvc("claim", storage_class="")])
    add("missing-class-bound", "1198-1217", [pod(0, claims=["claim"])], [True],
        pvcs=[pvc("claim", storage_class="missing-storage-class", volume_name="test-volume")],
        pvs=[pv("test-volume", storage_class="missing-storage-class")])
    add("missing-class-unbound", "1218-1229", [pod(0, claims=["claim"])], [False],
        pvcs=[pvc("claim", storage_class="missing-storage-class")])
    add("valid-pods-beside-invalid-pvc", "1230-1240", [pod(0, claims=["invalid"]), pod(1)], [False, True])
    add("valid-pods-beside-invalid-class", "1241-1253", [pod(0, claims=["claim"]), pod(1)], [False, True],
        pvcs=[pvc("claim", storage_class="invalid-storage-class")])
    add("valid-pods-beside-invalid-volume", "1254-1266", [pod(0, claims=["claim"]), pod(1)], [False, True],
        pvcs=[pvc("claim", volume_name="invalid-volume-name")])
    zone13 = [{"key": synth.ZONE, "operator": "In", "values": ["test-zone-1", "test-zone-3"]}]
    zone1 = [{"key": synth.ZONE, "operator": "In", "values": ["test-zone-1"]}]
    add("class-zones-unbound", "1267-1279", [pod(0, claims=["claim"], node_requirements=zone13)], ["test-zone-3"],
        pvcs=[pvc("claim", storage_class="my-storage-class")], scs=[SC])
    p = pod(0, ephemeral=["my-storage-class"], node_requirements=zone13)
    add("class-zones-unbound-ephemeral", "1280-1301", [p], ["test-zone-3"],
        pvcs=[pvc(ephemeral_claim(p), storage_class="my-storage-class")], scs=[SC])
    add("class-zones-incompatible", "1302-1313", [pod(0, claims=["claim"], node_requirements=zone1)], [False],
        pvcs=[pvc("claim", storage_class="my-storage-class")], scs=[SC])
    p = pod(0, ephemeral=["my-storage-class"], node_requirements=zone1)
    add("class-zones-incompatible-ephemeral", "1314-1334", [p], [False],
        pvcs=[pvc(ephemeral_claim(p), storage_class="my-storage-class")], scs=[SC])
    add("volume-zones-bound", "1335-1345", [pod(0, claims=["claim"])], ["test-zone-3"],
        pvcs=[pvc("claim", storage_class="my-storage-class", volume_name="pv-zone-3")],
        pvs=[pv("pv-zone-3", zones=["test-zone-3"])], scs=[SC])
    p = pod(0, ephemeral=["my-storage-class"])
    add("volume-zones-bound-ephemeral", "1346-1366", [p], ["test-zone-3"],
        pvcs=[pvc(ephemeral_claim(p), storage_class="my-storage-class", volume_name="pv-zone-3")],
        pvs=[pv("pv-zone-3", zones=["test-zone-3"])], scs=[SC])
    add("volume-zones-incompatible", "1367-1379", [pod(0, claims=["claim"], node_requirements=zone1)], [False],
        pvcs=[pvc("claim", storage_class="my-storage-class", volume_name="pv-zone-3")],
        pvs=[pv("pv-zone-3", zones=["test-zone-3"])], scs=[SC])
    p = pod(0, ephemeral=["my-storage-class"], node_requirements=zone1)
    add("volume-zones-incompatible-ephemeral", "1380-1402", [p], [False],
        pvcs=[pvc(ephemeral_claim(p), storage_class="my-storage-class", volume_name="pv-zone-3")],
        pvs=[pv("pv-zone-3", zones=["test-zone-3"])], scs=[SC])
    # the volume requirement is ANDed into every term: relaxing the first (unsatisfiable) term away keeps it
    p = pod(0, claims=["claim"],
            node_requirements=[{"key": "example.com/label", "operator": "In", "values": ["unsupported"]}],
            extra_terms=[{"matchExpressions": [{"key": synth.CT, "operator": "In", "values": ["on-demand"]}]}])
    add("volume-zone-not-relaxed-away", "1403-1435", [p], ["test-zone-3"],
        pvcs=[pvc("claim", storage_class="my-storage-class", volume_name="pv-zone-3")],
        pvs=[pv("pv-zone-3", zones=["test-zone-3"])], scs=[SC])
    return out


def check(scn, res):
    """res: canonical results.  The reference assertions: ExpectScheduled (+ node zone) / ExpectNotScheduled."""
    pods = scn["snapshot"]["pods"]
    idx = {p["metadata"]["name"]: i for i, p in enumerate(pods)}
    bad = []
    for name, want in scn["expect"].items():
        if name in scn["dropped"]:
            if want is not False:
                bad.append("%s dropped by GetPendingPods, want %s" % (name, want))
            continue
        i = idx[name]
        claims = [c for c in res["newNodeClaims"] if i in c["pods"]]
        on_node = any(i in n["pods"] for n in res["existingNodes"])
        scheduled = (bool(claims) or on_node) and str(i) not in res["podErrors"]
        if want is False:
            if scheduled:
                bad.append("%s scheduled, want unschedulable" % name)
            continue
        if not scheduled:
            bad.append("%s not scheduled (%s)" % (name, res["podErrors"].get(str(i))))
            continue
        if isinstance(want, str):
            zreq = [r for r in claims[0]["requirements"] if r.startswith(synth.ZONE + " ")]
            if zreq != ["%s In [%s]" % (synth.ZONE, want)]:
                bad.append("%s zone requirement %s, want %s" % (name, zreq, want))
    return bad


def main():
    fx = [{"name": s["name"], "source": s["source"], "dropped": s["dropped"], "expect": s["expect"]} for s in scenarios()]
    if "--write" in sys.argv:
        with open(os.path.join(HERE, "volume_topology_scenarios.json"), "w") as f:
            json.dump(fx, f, indent=1)
    print(json.dumps(fx, indent=1))


if __name__ == "__main__":
    main()
