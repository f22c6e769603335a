#!/usr/bin/env python3
"""Known-answer topology scenarios hand-transcribed from the reference's Go tests.

Source: pkg/controllers/provisioning/scheduling/topology_test.go (suite setup: suite_test.go:82-130,
the fake provider's default instance types fake/cloudprovider.go:177-214, and the Topology suite's
NodePool: test.NodePool with a capacity-type Exists requirement, topology_test.go:41-56).  Each
scenario is {"name", "source", "snapshot", "expect"}; `expect` holds the Go test's assertions:
  skew        : {"key", "selector"?, "counts"}: ExpectSkew (expectations.go:479-504) -- pods in
                namespace default matching the constraint's selector (nil: every pod), counted by the
                domain of the node they landed on -- as a multiset
  scheduled   : pod indices that must be scheduled;  unscheduled : pod indices that must not be
  one_node    : the listed pods share one node;  distinct : each listed pair lands on different nodes
New nodes get their labels from fake CloudProvider.Create (fake/cloudprovider.go:82-145): the
cheapest compatible instance type and its first available offering compatible with the claim's
zone / capacity-type requirements.  Run with --write to regenerate topology_scenarios.json.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "karpenter-sigs_amd"))
sys.path.insert(0, HERE)
from karpenter_amd import synth  # noqa: E402
from make_scenario_fixtures import default_instance_types  # noqa: E402

Z1, Z2, Z3 = "test-zone-1", "test-zone-2", "test-zone-3"
LABELS = {"test": "test"}
SRC = "pkg/controllers/provisioning/scheduling/topology_test.go:"


def pool(name="default", requirements=None, labels=None):
    reqs = requirements if requirements is not None else [{"key": synth.CT, "operator": "Exists"}]
    return synth.node_pool(name, limits={"cpu": "2000"}, requirements=reqs, labels=labels)


def tsc(key, max_skew=1, selector="labels", when="DoNotSchedule", min_domains=None):
    c = {"topologyKey": key, "whenUnsatisfiable": when, "maxSkew": max_skew}
    if selector == "labels":
        c["labelSelector"] = {"matchLabels": dict(LABELS)}
    elif selector is not None:
        c["labelSelector"] = selector
    if min_domains is not None:
        c["minDomains"] = min_domains
    return c


class PodFactory:
    def __init__(self):
        self.n = 0

    def __call__(self, count=1, labels=None, tscs=None, node_selector=None, cpu=None, anti_required=None,
                 anti_preferred=None, node_preferences=None, aff_required=None, aff_preferred=None, namespace="default",
                 node_requirements=None):
        out = []
        for _ in range(count):
            aff = {}
            if aff_required or aff_preferred:
                aff["podAffinity"] = {}
                if aff_required:
                    aff["podAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"] = aff_required
                if aff_preferred:
                    aff["podAffinity"]["preferredDuringSchedulingIgnoredDuringExecution"] = aff_preferred
            if node_requirements:
                aff["nodeAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": {
                    "nodeSelectorTerms": [{"matchExpressions": node_requirements}]}}
            if anti_required or anti_preferred:
                aff["podAntiAffinity"] = {}
                if anti_required:
                    aff["podAntiAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"] = anti_required
                if anti_preferred:
                    aff["podAntiAffinity"]["preferredDuringSchedulingIgnoredDuringExecution"] = anti_preferred
            if node_preferences:
                aff.setdefault("nodeAffinity", {})["preferredDuringSchedulingIgnoredDuringExecution"] = [
                    {"weight": 1, "preference": {"matchExpressions": node_preferences}}]
            p = synth.pod(self.n, cpu=cpu, labels=labels, node_selector=node_selector, affinity=aff or None,
                          namespace=namespace)
            p["metadata"]["labels"].pop("testing/cluster", None)  # test.Pod() sets no labels
            for k, v in (labels or {}).items():
                p["metadata"]["labels"][k] = v
            if tscs:
                p["spec"]["topologySpreadConstraints"] = tscs
            out.append(p)
            self.n += 1
        return out


def snapshot(pods, pools=None):
    its = default_instance_types()
    pools = pools or [pool()]
    return {
        "wellKnownLabels": synth.FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": {p["metadata"]["name"]: list(range(len(its))) for p in pools},
        "nodeClaimTemplates": pools,
        "nodePools": pools,
        "stateNodes": [],
        "daemonSetPods": [],
        "pods": pods,
    }


def scenarios():
    out = []

    def add(name, line, pods, expect, pools=None):
        out.append({"name": name, "source": SRC + line, "snapshot": snapshot(pods, pools), "expect": expect})

    zone = synth.ZONE
    # Zonal
    P = PodFactory()
    add("zonal-match-labels", "93-105", P(4, LABELS, [tsc(zone)]), {"skew": {"key": zone, "counts": [1, 1, 2]}})
    P = PodFactory()
    expr = {"matchExpressions": [{"key": "test", "operator": "In", "values": ["test"]}]}
    add("zonal-match-expressions", "106-126", P(4, LABELS, [tsc(zone, selector=expr)]),
        {"skew": {"key": zone, "selector": expr, "counts": [1, 1, 2]}})
    P = PodFactory()
    add("zonal-nodepool-constraints", "127-141", P(4, LABELS, [tsc(zone)]),
        {"skew": {"key": zone, "counts": [1, 1, 2]}},
        [pool(requirements=[{"key": zone, "operator": "In", "values": [Z1, Z2, Z3]}])])
    P = PodFactory()
    add("zonal-subset-requirements", "142-157", P(4, LABELS, [tsc(zone)]),
        {"skew": {"key": zone, "counts": [2, 2]}},
        [pool(requirements=[{"key": zone, "operator": "In", "values": [Z1, Z2]}])])
    P = PodFactory()
    add("zonal-subset-labels", "158-172", P(4, LABELS, [tsc(zone)]), {"skew": {"key": zone, "counts": [4]}},
        [pool(labels={zone: Z1})])
    P = PodFactory()
    add("zonal-subset-requirements-and-labels", "173-188", P(4, LABELS, [tsc(zone)]),
        {"skew": {"key": zone, "counts": [4]}},
        [pool(requirements=[{"key": zone, "operator": "In", "values": [Z1, Z2]}], labels={zone: Z1})])
    P = PodFactory()
    add("zonal-subset-labels-across-nodepools", "189-216", P(4, LABELS, [tsc(zone)]),
        {"skew": {"key": zone, "counts": [2, 2]}},
        [pool(requirements=[{"key": zone, "operator": "In", "values": [Z1, Z2]}], labels={zone: Z1}),
         pool("nodepool-2", requirements=[], labels={zone: Z2})])
    P = PodFactory()
    add("zonal-no-label-selector", "430-441", P(1, None, [tsc(zone, selector=None)]),
        {"skew": {"key": zone, "selector": None, "counts": [1]}})
    P = PodFactory()
    add("interdependent-selectors", "442-466", P(5, None, [tsc(synth.HOSTNAME)]), {"one_node": [0, 1, 2, 3, 4]})
    P = PodFactory()
    add("min-domains-unsatisfied", "467-486", P(3, LABELS, [tsc(zone, min_domains=3)]),
        {"skew": {"key": zone, "counts": [1, 1]}},
        [pool(requirements=[{"key": zone, "operator": "In", "values": [Z1, Z2]}])])
    P = PodFactory()
    add("min-domains-equal", "487-506", P(11, LABELS, [tsc(zone, min_domains=3)]),
        {"skew": {"key": zone, "counts": [4, 4, 3]}},
        [pool(requirements=[{"key": zone, "operator": "In", "values": [Z1, Z2, Z3]}])])
    P = PodFactory()
    add("min-domains-greater", "507-526", P(11, LABELS, [tsc(zone, min_domains=2)]),
        {"skew": {"key": zone, "counts": [4, 4, 3]}},
        [pool(requirements=[{"key": zone, "operator": "In", "values": [Z1, Z2, Z3]}])])
    # Hostname
    P = PodFactory()
    add("hostname-balance", "530-542", P(4, LABELS, [tsc(synth.HOSTNAME)]),
        {"skew": {"key": synth.HOSTNAME, "counts": [1, 1, 1, 1]}})
    P = PodFactory()
    add("hostname-max-skew-4", "543-555", P(4, LABELS, [tsc(synth.HOSTNAME, max_skew=4)]),
        {"skew": {"key": synth.HOSTNAME, "counts": [4]}})
    # Capacity type
    P = PodFactory()
    add("capacity-type-balance", "638-650", P(4, LABELS, [tsc(synth.CT)]),
        {"skew": {"key": synth.CT, "counts": [2, 2]}})
    P = PodFactory()
    add("capacity-type-nodepool-constraints", "651-665", P(4, LABELS, [tsc(synth.CT)]),
        {"skew": {"key": synth.CT, "counts": [2, 2]}},
        [pool(requirements=[{"key": synth.CT, "operator": "In", "values": ["spot", "on-demand"]}])])
    # Unknown key
    P = PodFactory()
    add("ignore-unknown-topology-keys", "58-74", P(1, LABELS, [tsc("unknown")]) + P(1),
        {"unscheduled": [0], "scheduled": [1]})
    # Zonal + node affinity
    P = PodFactory()
    add("spread-limited-by-node-selector", "1196-1221",
        P(5, LABELS, [tsc(zone)], node_selector={zone: Z1}) + P(10, LABELS, [tsc(zone)], node_selector={zone: Z2}),
        {"skew": {"key": zone, "counts": [5, 10]}})
    P = PodFactory()
    add("spread-not-limited-by-preferred-affinity", "1288-1308",
        P(6, LABELS, [tsc(zone)], node_preferences=[{"key": zone, "operator": "In", "values": [Z1, Z2]}]),
        {"skew": {"key": zone, "counts": [2, 2, 2]}})
    # Anti-affinity
    sec = {"security": "s2"}
    term = lambda key: {"labelSelector": {"matchLabels": dict(sec)}, "topologyKey": key}  # noqa: E731
    P = PodFactory()
    add("anti-affinity-preferred-violation", "1667-1699",
        P(3, LABELS, [tsc(zone)]) + P(10, anti_preferred=[{"weight": 50, "podAffinityTerm": {
            "labelSelector": {"matchLabels": dict(LABELS)}, "topologyKey": zone}}]),
        {"scheduled": list(range(3, 13))})
    P = PodFactory()
    add("anti-affinity-hostname-separates", "1700-1721", P(1, anti_required=[term(synth.HOSTNAME)]) + P(1, sec),
        {"scheduled": [0, 1], "distinct": [[0, 1]]})
    P = PodFactory()
    add("anti-affinity-zone", "1722-1760",
        P(1, sec, node_selector={zone: Z1}, cpu="2") + P(1, sec, node_selector={zone: Z2}, cpu="2") +
        P(1, sec, node_selector={zone: Z3}, cpu="2") + P(1, anti_required=[term(zone)]),
        {"scheduled": [0, 1, 2], "unscheduled": [3]})
    P = PodFactory()
    add("anti-affinity-zone-other-schedules-first", "1761-1782", P(1, sec, cpu="2") + P(1, anti_required=[term(zone)]),
        {"scheduled": [0], "unscheduled": [1]})
    P = PodFactory()
    pref = [{"weight": 10, "podAffinityTerm": term(zone)}]
    add("anti-affinity-preferred-zone-inverse", "1826-1865",
        P(1, node_selector={zone: Z1}, cpu="2", anti_preferred=pref) +
        P(1, node_selector={zone: Z2}, cpu="2", anti_preferred=pref) +
        P(1, node_selector={zone: Z3}, cpu="2", anti_preferred=pref) + P(1, sec),
        {"scheduled": [0, 1, 2, 3]})
    P = PodFactory()
    add("anti-affinity-zone-inverse", "1866-1901",
        P(1, node_selector={zone: Z1}, cpu="2", anti_required=[term(zone)]) +
        P(1, node_selector={zone: Z2}, cpu="2", anti_required=[term(zone)]) +
        P(1, node_selector={zone: Z3}, cpu="2", anti_required=[term(zone)]) + P(1, sec),
        {"scheduled": [0, 1, 2], "unscheduled": [3]})
    # Pod affinity (topology_test.go "Pod Affinity/Anti-Affinity"); single-batch assertions only
    arch, host = synth.ARCH, synth.HOSTNAME
    P = PodFactory()
    add("affinity-arch", "1426-1468",
        P(1, sec, [tsc(host, selector={"matchLabels": dict(sec)})], cpu="2", node_selector={arch: "arm64"}) +
        P(1, sec, [tsc(host, selector={"matchLabels": dict(sec)})], cpu="1", aff_required=[term(arch)]),
        {"scheduled": [0, 1], "distinct": [[0, 1]], "same_label": [{"key": arch, "pods": [0, 1]}]})
    P = PodFactory()
    add("self-affinity-hostname", "1469-1492", P(3, sec, aff_required=[term(host)]),
        {"scheduled": [0, 1, 2], "one_node": [0, 1, 2]})
    P = PodFactory()
    add("self-affinity-hostname-first-domain", "1493-1534", P(10, sec, aff_required=[term(host)]),
        {"count_scheduled": 5, "nodes_used": 1})
    P = PodFactory()
    add("self-affinity-zone", "1579-1602", P(3, sec, aff_required=[term(zone)]),
        {"scheduled": [0, 1, 2], "one_node": [0, 1, 2]})
    P = PodFactory()
    add("self-affinity-zone-constrained", "1603-1633",
        P(3, sec, aff_required=[term(zone)], node_requirements=[{"key": zone, "operator": "In", "values": [Z3]}]),
        {"scheduled": [0, 1, 2], "one_node": [0, 1, 2], "label_value": {"key": zone, "value": Z3, "pods": [0, 1, 2]}})
    P = PodFactory()
    add("affinity-preferred-violation", "1634-1666",
        P(10, LABELS, [tsc(host)]) + P(1, aff_preferred=[{"weight": 50, "podAffinityTerm": term(host)}]),
        {"scheduled": [10]})
    P = PodFactory()
    cons = tsc(host)
    add("affinity-preference-vs-required-spread", "2034-2068",
        P(3, LABELS, [cons], aff_preferred=[{"weight": 50, "podAffinityTerm": term(host)}]) + P(1, sec),
        {"scheduled": [0, 1, 2, 3], "skew": {"key": host, "counts": [1, 1, 1]}})
    P = PodFactory()
    add("affinity-to-missing-pod", "2114-2130", P(10, aff_required=[term(zone)]),
        {"unscheduled": list(range(10))})
    P = PodFactory()
    add("affinity-zone-unconstrained-target", "2131-2163", P(10, aff_required=[term(zone)]) + P(1, sec),
        {"unscheduled": list(range(10)), "scheduled": [10], "skew": {"key": zone, "selector": None, "counts": [1]}})
    P = PodFactory()
    add("affinity-zone-constrained-target", "2164-2192",
        P(10, aff_required=[term(zone)]) +
        P(1, sec, node_requirements=[{"key": zone, "operator": "In", "values": [Z1]}]),
        {"scheduled": list(range(11)), "skew": {"key": zone, "selector": None, "counts": [11]}})
    P = PodFactory()
    db, web, cache, ui = ({"type": t, "spread": "spread"} for t in ("db", "web", "cache", "ui"))
    dep = lambda lab: [{"labelSelector": {"matchLabels": dict(lab)}, "topologyKey": host}]  # noqa: E731
    add("multiple-dependent-affinities", "2193-2227",
        P(1, db) + P(1, web, aff_required=dep(db)) + P(1, cache, aff_required=dep(web)) + P(1, ui, aff_required=dep(cache)),
        {"scheduled": [0, 1, 2, 3]})
    P = PodFactory()
    add("unsatisfiable-dependencies", "2228-2243", P(1, db, aff_required=dep(web)), {"unscheduled": [0]})
    P = PodFactory()
    add("affinity-namespace-no-match", "2244-2281",
        P(10, LABELS, [tsc(host)]) + P(1, sec, namespace="other-ns-no-match") + P(1, aff_required=[term(host)]),
        {"scheduled": [10], "unscheduled": [11]})
    P = PodFactory()
    t_ns = {"labelSelector": {"matchLabels": dict(sec)}, "namespaces": ["other-ns-list"], "topologyKey": host}
    add("affinity-namespace-list", "2282-2320",
        P(10, LABELS, [tsc(host)]) + P(1, sec, namespace="other-ns-list") + P(1, aff_required=[t_ns]),
        {"scheduled": [10, 11], "one_node": [10, 11]})
    # the envtest cluster's namespaces plus the one the test applies (topology_test.go:2331)
    namespaces = [{"name": n} for n in ("default", "kube-system", "kube-public", "kube-node-lease")] + [
        {"name": "empty-ns-selector", "labels": {"foo": "bar"}}]
    P = PodFactory()
    t_sel = {"labelSelector": {"matchLabels": dict(sec)}, "namespaceSelector": {"matchLabels": {}}, "topologyKey": host}
    add("affinity-namespace-empty-selector", "2321-2361",
        P(10, LABELS, [tsc(host)]) + P(1, sec, namespace="empty-ns-selector") + P(1, aff_required=[t_sel]),
        {"scheduled": [10, 11], "one_node": [10, 11]})
    out[-1]["snapshot"]["namespaces"] = namespaces
    # the same test with a selector that picks the namespace by label, and one that matches nothing
    P = PodFactory()
    t_lab = {"labelSelector": {"matchLabels": dict(sec)}, "namespaceSelector": {"matchLabels": {"foo": "bar"}},
             "topologyKey": host}
    add("affinity-namespace-label-selector", "2321-2361",
        P(10, LABELS, [tsc(host)]) + P(1, sec, namespace="empty-ns-selector") + P(1, aff_required=[t_lab]),
        {"scheduled": [10, 11], "one_node": [10, 11]})
    out[-1]["snapshot"]["namespaces"] = namespaces
    P = PodFactory()
    t_none = {"labelSelector": {"matchLabels": dict(sec)},
              "namespaceSelector": {"matchExpressions": [{"key": "foo", "operator": "In", "values": ["baz"]}]},
              "topologyKey": host}
    add("affinity-namespace-selector-no-match", "2244-2281",
        P(10, LABELS, [tsc(host)]) + P(1, sec, namespace="empty-ns-selector") + P(1, aff_required=[t_none]),
        {"scheduled": [10], "unscheduled": [11]})
    out[-1]["snapshot"]["namespaces"] = namespaces
    return out


def _req_values(claim, key):
    for r in claim["requirements"]:
        parts = r.split(" ")
        if parts[0] == key and parts[1] == "In":
            return r[r.index("[") + 1:r.index("]")].split(" ")
    return None


def node_labels(claim, snap):
    """fake CloudProvider.Create: cheapest compatible instance type, first compatible offering."""
    its = {it["name"]: it for it in snap["instanceTypes"]}
    zones, cts = _req_values(claim, synth.ZONE), _req_values(claim, synth.CT)
    ok = lambda o: (o.get("available", True) and (zones is None or o["zone"] in zones)  # noqa: E731
                    and (cts is None or o["capacityType"] in cts))
    best = None
    for name in claim["instanceTypeOptions"]:
        prices = [o["price"] for o in its[name]["offerings"] if ok(o)]
        if prices and (best is None or min(prices) < best[0]):
            best = (min(prices), name)
    it = its[best[1]]
    labels = {}
    for r in it["requirements"]:
        if r["operator"] == "In" and r.get("values"):
            labels[r["key"]] = r["values"][0]
    for o in it["offerings"]:
        if ok(o):
            labels[synth.ZONE], labels[synth.CT] = o["zone"], o["capacityType"]
            break
    return labels


def node_of(res):
    """pod index -> claim index"""
    out = {}
    for ci, c in enumerate(res["newNodeClaims"]):
        for p in c["pods"]:
            out[p] = ci
    return out


def selector_matches(sel, labels):
    if sel is None:
        return True
    for k, v in sel.get("matchLabels", {}).items():
        if labels.get(k) != v:
            return False
    for e in sel.get("matchExpressions", []):
        has, val = e["key"] in labels, labels.get(e["key"])
        if e["operator"] == "In" and not (has and val in e["values"]):
            return False
        if e["operator"] == "NotIn" and has and val in e["values"]:
            return False
        if e["operator"] == "Exists" and not has:
            return False
        if e["operator"] == "DoesNotExist" and has:
            return False
    return True


def check(scn, res):
    """Violated expectations of a scenario given canonical Solve results (empty list = pass)."""
    exp, snap = scn["expect"], scn["snapshot"]
    bad = []
    where = node_of(res)
    scheduled = {p for p in range(len(snap["pods"])) if str(p) not in res["podErrors"]}
    for p in exp.get("scheduled", []):
        if p not in scheduled:
            bad.append("pod %d not scheduled" % p)
    for p in exp.get("unscheduled", []):
        if p in scheduled:
            bad.append("pod %d scheduled" % p)
    if "one_node" in exp and len({where.get(p) for p in exp["one_node"]}) != 1:
        bad.append("pods %s on several nodes" % exp["one_node"])
    for a, b in exp.get("distinct", []):
        if where.get(a) == where.get(b):
            bad.append("pods %d and %d share a node" % (a, b))
    if "count_scheduled" in exp and len(scheduled) != exp["count_scheduled"]:
        bad.append("%d scheduled, want %d" % (len(scheduled), exp["count_scheduled"]))
    if "nodes_used" in exp and len(res["newNodeClaims"]) != exp["nodes_used"]:
        bad.append("%d nodes, want %d" % (len(res["newNodeClaims"]), exp["nodes_used"]))
    for same in exp.get("same_label", []):
        vals = {node_labels(res["newNodeClaims"][where[p]], snap).get(same["key"]) for p in same["pods"] if p in where}
        if len(vals) != 1:
            bad.append("pods %s on %s values %s" % (same["pods"], same["key"], sorted(map(str, vals))))
    if "label_value" in exp:
        lv = exp["label_value"]
        for p in lv["pods"]:
            if p in where and node_labels(res["newNodeClaims"][where[p]], snap).get(lv["key"]) != lv["value"]:
                bad.append("pod %d not on %s=%s" % (p, lv["key"], lv["value"]))
    if "skew" in exp:
        sk = exp["skew"]
        sel = sk.get("selector", {"matchLabels": LABELS}) if "selector" in sk else {"matchLabels": LABELS}
        counts = {}
        for ci, c in enumerate(res["newNodeClaims"]):
            labels = node_labels(c, snap)
            for p in c["pods"]:
                if not selector_matches(sel, snap["pods"][p]["metadata"].get("labels", {})):
                    continue
                dom = "node-%d" % ci if sk["key"] == synth.HOSTNAME else labels.get(sk["key"])
                if dom is not None:
                    counts[dom] = counts.get(dom, 0) + 1
        if sorted(counts.values()) != sorted(sk["counts"]):
            bad.append("skew %s != %s" % (sorted(counts.values()), sorted(sk["counts"])))
    return bad


if __name__ == "__main__":
    if "--write" in sys.argv:
        data = [{"name": s["name"], "source": s["source"], "expect": s["expect"]} for s in scenarios()]
        with open(os.path.join(HERE, "topology_scenarios.json"), "w") as f:
            json.dump(data, f, indent=1)
        print("wrote %d scenarios" % len(data))
