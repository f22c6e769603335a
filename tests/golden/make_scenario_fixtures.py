#!/usr/bin/env python3
"""Known-answer scheduling scenarios hand-transcribed from the reference's Go tests into snapshots.

Each scenario is {"name", "source", "snapshot", "expect"} where `expect` holds the reference test's
assertions:
  nodes        : number of distinct nodes (new NodeClaims) the pods land on
  type         : instance type the fake cloud provider launches for every claim
                 (fake/cloudprovider.go:96-141: cheapest option by available-offering price)
  types_differ : the claims launch different instance types
  scheduled    : all pods scheduled (True) / the listed pod indices unschedulable
Sources: pkg/controllers/provisioning/scheduling/suite_test.go (Binpacking :1462-1766,
Instance Type Compatibility :1358-1458), suite setup :82-130 (fake.NewCloudProvider default
instance types, cloudprovider.go:177-214; test.NodePool with capacity-type requirements and the
default cpu limit 2000, pkg/test/nodepool.go:43-45).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "karpenter-sigs_amd"))
from karpenter_amd import synth  # noqa: E402


def default_instance_types():
    """fake.CloudProvider.GetInstanceTypes defaults (fake/cloudprovider.go:177-214)."""
    return [
        synth.fake_instance_type("default-instance-type", 4, 4, pods=5),
        synth.fake_instance_type("small-instance-type", 2, 2, pods=5),
        synth.fake_instance_type("gpu-vendor-instance-type", 4, 4, pods=5, extra_capacity={"fake.com/vendor-a": "2"}),
        synth.fake_instance_type("gpu-vendor-b-instance-type", 4, 4, pods=5, extra_capacity={"fake.com/vendor-b": "2"}),
        synth.fake_instance_type("arm-instance-type", 16, 128, pods=5, arch="arm64",
                                 oses=("darwin", "ios", "linux", "windows")),
        synth.fake_instance_type("single-pod-instance-type", 4, 4, pods=1),
    ]


def suite_nodepool(name="default"):
    # suite_test.go:112-129 + test.NodePool defaults (limits cpu: 2000)
    return synth.node_pool(name, limits={"cpu": "2000"},
                           requirements=[{"key": synth.CT, "operator": "In", "values": ["spot", "on-demand"]}])


def snapshot(pods, its=None):
    its = its if its is not None else default_instance_types()
    np_obj = suite_nodepool()
    return {
        "wellKnownLabels": synth.FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": {"default": list(range(len(its)))},
        "nodeClaimTemplates": [np_obj],
        "nodePools": [np_obj],
        "stateNodes": [],
        "daemonSetPods": [],
        "pods": pods,
    }


def pods(n, start=0, **kw):
    out = []
    for i in range(n):
        out.append(synth.pod(start + i, **kw))
    return out


def with_requests(p, req, limits=None):
    p["spec"]["containers"][0]["resources"] = {"requests": req}
    if limits:
        p["spec"]["containers"][0]["resources"]["limits"] = limits
    return p


def scenarios():
    S = []
    src = "pkg/controllers/provisioning/scheduling/suite_test.go"
    S.append({"name": "small-pod-smallest-instance", "source": src + ":1463-1474",
              "snapshot": snapshot([synth.pod(0, mem="100M")]),
              "expect": {"nodes": 1, "type": "small-instance-type", "scheduled": True}})
    S.append({"name": "small-pod-smallest-possible", "source": src + ":1475-1486",
              "snapshot": snapshot([synth.pod(0, mem="2000M")]),
              "expect": {"nodes": 1, "type": "small-instance-type", "scheduled": True}})
    p = synth.pod(0, cpu="1")
    p["spec"]["overhead"] = {"cpu": "2"}  # RuntimeClass PodFixed overhead applied at admission
    S.append({"name": "runtime-class-overhead", "source": src + ":1487-1514",
              "snapshot": snapshot([p]), "expect": {"nodes": 1, "type": "default-instance-type", "scheduled": True}})
    S.append({"name": "5x10M-one-small-node", "source": src + ":1515-1533",
              "snapshot": snapshot(pods(5, mem="10M")),
              "expect": {"nodes": 1, "type": "small-instance-type", "scheduled": True}})
    S.append({"name": "40x1.8G-twenty-nodes", "source": src + ":1534-1553",
              "snapshot": snapshot(pods(40, mem="1.8G", node_selector={synth.ARCH: "amd64"})),
              "expect": {"nodes": 20, "type": "default-instance-type", "scheduled": True}})
    S.append({"name": "40-large-20-small-pack", "source": src + ":1554-1585",
              "snapshot": snapshot(pods(40, mem="1.8G", node_selector={synth.ARCH: "amd64"}) +
                                   pods(20, start=40, mem="400M", node_selector={synth.ARCH: "amd64"})),
              "expect": {"nodes": 20, "type": "default-instance-type", "scheduled": True}})
    S.append({"name": "pack-tightly-fake5", "source": src + ":1586-1611",
              "snapshot": snapshot([synth.pod(0, cpu="4.5"), synth.pod(1, cpu="1")], its=synth.fake_instance_types(5)),
              "expect": {"nodes": 2, "types_differ": True, "scheduled": True}})
    S.append({"name": "zero-quantity-resource", "source": src + ":1612-1623",
              "snapshot": snapshot([with_requests(synth.pod(0), {"foo.com/weird-resources": "0"},
                                                  {"foo.com/weird-resources": "0"})]),
              "expect": {"nodes": 1, "scheduled": True}})
    S.append({"name": "2Ti-unschedulable", "source": src + ":1624-1634",
              "snapshot": snapshot([synth.pod(0, mem="2Ti")]), "expect": {"nodes": 0, "scheduled": [0]}})
    S.append({"name": "pod-limit-per-node", "source": src + ":1635-1656",
              "snapshot": snapshot(pods(25, cpu="1m", mem="1m", node_selector={synth.ARCH: "amd64"})),
              "expect": {"nodes": 5, "type": "small-instance-type", "scheduled": True}})
    p = synth.pod(0, cpu="1", mem="1Gi")
    p["spec"]["initContainers"] = [{"name": "init", "resources": {"requests": {"cpu": "2", "memory": "1Gi"}}}]
    S.append({"name": "init-container-max", "source": src + ":1657-1677",
              "snapshot": snapshot([p]), "expect": {"nodes": 1, "type": "default-instance-type", "scheduled": True}})
    p = synth.pod(0, cpu="1", mem="1Gi")
    p["spec"]["initContainers"] = [{"name": "init", "resources": {"requests": {"cpu": "2", "memory": "1Ti"}}}]
    S.append({"name": "init-container-too-big", "source": src + ":1678-1697",
              "snapshot": snapshot([p]), "expect": {"nodes": 0, "scheduled": [0]}})
    # Provider Specific Labels (suite_test.go:1405-1458): fake.InstanceTypes(5) with size/special labels
    its5 = synth.fake_instance_types(5)
    S.append({"name": "it-filter-by-labels", "source": src + ":1406-1418",
              "snapshot": snapshot([synth.pod(0, node_selector={"size": "large"}),
                                    synth.pod(1, node_selector={"size": "small"})], its=its5),
              "expect": {"nodes": 2, "pod_types": {"0": "fake-it-4", "1": "fake-it-0"}, "scheduled": True}})
    S.append({"name": "it-incompatible-labels", "source": src + ":1419-1435",
              "snapshot": snapshot([synth.pod(0, node_selector={"size": "large", synth.IT_LABEL: "fake-it-0"}),
                                    synth.pod(1, node_selector={"size": "small", synth.IT_LABEL: "fake-it-4"})],
                                   its=its5),
              "expect": {"nodes": 0, "scheduled": [0, 1]}})
    p = synth.pod(0, affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchExpressions": [{"key": "special", "operator": "Exists"}]}]}}})
    S.append({"name": "it-optional-label-exists", "source": src + ":1436-1447",
              "snapshot": snapshot([p], its=its5), "expect": {"nodes": 1, "type": "fake-it-4", "scheduled": True}})
    p = synth.pod(0, affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchExpressions": [{"key": "special", "operator": "DoesNotExist"}]}]}}})
    snap = snapshot([p], its=its5)
    snap["nodeClaimTemplates"] = [synth.node_pool("default", limits={"cpu": "2000"})]  # plain test.NodePool()
    snap["nodePools"] = snap["nodeClaimTemplates"]
    S.append({"name": "it-optional-label-disallowed", "source": src + ":1448-1458",
              "snapshot": snap, "expect": {"nodes": 1, "type": "fake-it-0", "scheduled": True}})
    return S


def main():
    out = scenarios()
    with open(os.path.join(HERE, "scenarios.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("%d scenarios" % len(out))


if __name__ == "__main__":
    main()
