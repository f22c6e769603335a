"""Synthetic snapshots shaped like the reference's own test fixtures (BASELINE.json configs).

Mirrors pkg/cloudprovider/fake/instancetype.go (InstanceTypes(n), NewInstanceType,
priceFromResources), pkg/test (NodePool(), Pod()) and
pkg/controllers/provisioning/scheduling/scheduling_benchmark_test.go (makeDiversePods).  Go's
math/rand stream is not reproducible here, so distributions match the reference while the sequence
comes from numpy's PCG64 with the stated seed.
"""
import numpy as np

ZONE = "topology.kubernetes.io/zone"
CT = "karpenter.sh/capacity-type"
ARCH = "kubernetes.io/arch"
OS = "kubernetes.io/os"
IT_LABEL = "node.kubernetes.io/instance-type"
NODEPOOL = "karpenter.sh/nodepool"
HOSTNAME = "kubernetes.io/hostname"
WELL_KNOWN = [NODEPOOL, ZONE, "topology.kubernetes.io/region", IT_LABEL, ARCH, OS, CT,
              "node.kubernetes.io/windows-build"]
# fake/instancetype.go:42-48 — linking the fake provider inserts these into WellKnownLabels
FAKE_WELL_KNOWN = WELL_KNOWN + ["size", "special", "integer"]
GI = 1 << 30


def price_from_resources(cpu, mem_bytes, gpus=0):  # fake/instancetype.go:177-189
    return 0.1 * cpu + 0.1 * mem_bytes / 1e9 + 1.0 * gpus


def fake_instance_type(name, cpu, mem_gi, pods=None, arch="amd64", oses=("darwin", "linux", "windows"),
                       offerings=None, extra_capacity=None):
    """fake.NewInstanceType (instancetype.go:50-110) with integer cpu and Gi memory."""
    mem_bytes = mem_gi * GI
    price = price_from_resources(cpu, mem_bytes, len(extra_capacity or {}))
    if offerings is None:
        offerings = [
            {"capacityType": "spot", "zone": "test-zone-1", "price": price, "available": True},
            {"capacityType": "spot", "zone": "test-zone-2", "price": price, "available": True},
            {"capacityType": "on-demand", "zone": "test-zone-1", "price": price, "available": True},
            {"capacityType": "on-demand", "zone": "test-zone-2", "price": price, "available": True},
            {"capacityType": "on-demand", "zone": "test-zone-3", "price": price, "available": True},
        ]
    avail = [o for o in offerings if o.get("available", True)]
    large = cpu > 4 and mem_gi > 8
    reqs = [
        {"key": IT_LABEL, "operator": "In", "values": [name]},
        {"key": ARCH, "operator": "In", "values": [arch]},
        {"key": OS, "operator": "In", "values": sorted(oses)},
        {"key": ZONE, "operator": "In", "values": sorted({o["zone"] for o in avail})},
        {"key": CT, "operator": "In", "values": sorted({o["capacityType"] for o in avail})},
        {"key": "size", "operator": "In", "values": ["large" if large else "small"]},
        ({"key": "special", "operator": "In", "values": ["optional"]} if large
         else {"key": "special", "operator": "DoesNotExist"}),
        {"key": "integer", "operator": "In", "values": [str(cpu)]},
    ]
    cap = {"cpu": str(cpu), "memory": "%dGi" % mem_gi, "pods": str(pods if pods is not None else 5)}
    if extra_capacity:
        cap.update(extra_capacity)
    return {"name": name, "requirements": reqs, "offerings": offerings, "capacity": cap,
            "overhead": {"kubeReserved": {"cpu": "100m", "memory": "10Mi"}}}


def fake_instance_types(n):
    """fake.InstanceTypes(n) (instancetype.go:153-167): i+1 cpu, 2(i+1)Gi, 10(i+1) pods."""
    return [fake_instance_type("fake-it-%d" % i, i + 1, 2 * (i + 1), pods=10 * (i + 1)) for i in range(n)]


def node_pool(name, weight=None, limits=None, requirements=None, taints=None, labels=None):
    """test.NodePool() (pkg/test/nodepool.go:33-61) as a NodePool JSON object."""
    lab = {"testing/cluster": "unspecified"}
    lab.update(labels or {})
    spec = {"template": {"metadata": {"labels": lab},
                         "spec": {"requirements": requirements or [], "taints": taints or []}}}
    if weight is not None:
        spec["weight"] = weight
    if limits is not None:
        spec["limits"] = limits
    return {"metadata": {"name": name}, "spec": spec}


def pod(i, cpu=None, mem=None, labels=None, node_selector=None, affinity=None, tolerations=None,
        namespace="default", uid=None, extra=None):
    """test.Pod() (pkg/test/pods.go:72-150) with a unique UID (queue.go keys staleness by UID)."""
    lab = {"testing/cluster": "unspecified"}
    lab.update(labels or {})
    req = {}
    if cpu is not None:
        req["cpu"] = cpu
    if mem is not None:
        req["memory"] = mem
    spec = {"containers": [{"name": "c", "resources": {"requests": req}}]}
    if node_selector:
        spec["nodeSelector"] = node_selector
    if affinity:
        spec["affinity"] = affinity
    if tolerations:
        spec["tolerations"] = tolerations
    if extra:
        spec.update(extra)
    return {"metadata": {"name": "pod-%06d" % i, "namespace": namespace, "uid": uid or "pod-uid-%06d" % i,
                         "labels": lab},
            "spec": spec,
            "status": {"conditions": [{"type": "PodScheduled", "reason": "Unschedulable", "status": "False"}]}}


CPU_CHOICES = ["100m", "250m", "500m", "1000m", "1500m"]           # scheduling_benchmark_test.go:283-286
MEM_CHOICES = ["100Mi", "256Mi", "512Mi", "1024Mi", "2048Mi", "4096Mi"]  # :278-281
LABEL_VALUES = ["a", "b", "c", "d", "e", "f", "g"]                  # :273-276


def make_diverse_pods(count, rng):
    """makeDiversePods (scheduling_benchmark_test.go:184-196)."""
    pods = []

    def res():
        return CPU_CHOICES[rng.integers(len(CPU_CHOICES))], MEM_CHOICES[rng.integers(len(MEM_CHOICES))]

    def generic(n):
        for _ in range(n):
            lab = {"my-label": LABEL_VALUES[rng.integers(7)]}
            c, m = res()
            pods.append((lab, c, m, None))

    def spread(n, key):
        for _ in range(n):
            lab = {"my-label": LABEL_VALUES[rng.integers(7)]}
            sel = {"my-label": LABEL_VALUES[rng.integers(7)]}
            c, m = res()
            pods.append((lab, c, m, {"topologySpreadConstraints": [
                {"maxSkew": 1, "topologyKey": key, "whenUnsatisfiable": "DoNotSchedule",
                 "labelSelector": {"matchLabels": sel}}]}))

    def affinity(n, key):
        for _ in range(n):
            lab = {"my-affininity": LABEL_VALUES[rng.integers(7)]}
            sel = {"my-affininity": LABEL_VALUES[rng.integers(7)]}
            c, m = res()
            pods.append((lab, c, m, {"affinity": {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchLabels": sel}, "topologyKey": key}]}}}))

    generic(count // 7)
    spread(count // 7, ZONE)
    spread(count // 7, HOSTNAME)
    affinity(count // 7, HOSTNAME)
    affinity(count // 7, ZONE)
    generic(count - len(pods))
    out = []
    for i, (lab, c, m, extra) in enumerate(pods):
        p = pod(i, cpu=c, mem=m, labels=lab)
        if extra:
            p["spec"].update(extra)
        out.append(p)
    return out


def benchmark_snapshot(n_pods, n_its=400, seed=42, diverse=True, literal=False):
    """BenchmarkScheduling (scheduling_benchmark_test.go:116-182): one template from test.NodePool(),
    no NodePools (so no limits), empty Topology, fake.InstanceTypes(n_its).
    literal: the benchmark's pods exactly as test.Pod() builds them without an apiserver: no UID and a
    zero CreationTimestamp (pkg/test/pods.go, metadata.go), so NewQueue breaks cpu/memory ties with
    sort.Slice's tie order and every pod shares the staleness key "" (queue.go:38,54-69)."""
    rng = np.random.default_rng(seed)
    its = fake_instance_types(n_its)
    np_obj = node_pool("default-pool")
    if diverse:
        pods = make_diverse_pods(n_pods, rng)
    else:
        pods = []
        for i in range(n_pods):
            pods.append(pod(i, cpu=CPU_CHOICES[rng.integers(5)], mem=MEM_CHOICES[rng.integers(6)],
                            labels={"my-label": LABEL_VALUES[rng.integers(7)]}))
    if literal:
        for p in pods:
            p["metadata"].pop("uid", None)
    return {
        "wellKnownLabels": FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": {"default-pool": list(range(n_its))},
        "nodeClaimTemplates": [np_obj],
        "nodePools": [],
        "stateNodes": [],
        "daemonSetPods": [],
        "pods": pods,
        "emptyTopology": True,  # &scheduling.Topology{} (scheduling_benchmark_test.go:124)
    }


def config1(seed=42, literal=False):
    """C1: BenchmarkScheduling2000 — makeDiversePods(2000) x fake.InstanceTypes(400).
    literal=True: the benchmark's own pods (empty UIDs, zero timestamps)."""
    return benchmark_snapshot(2000, 400, seed, diverse=True, literal=literal)


def config2(n_pods=50000, seed=42):
    """C2: 50k resource-only pods x 400 fake instance types, 1 template, no limits."""
    return benchmark_snapshot(n_pods, 400, seed, diverse=False)


def _fmt_time(sec):
    import datetime
    return datetime.datetime.fromtimestamp(int(sec), tz=datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


NOW = 1760000000  # fixed "now" for lifetimeRemaining (types.go:136-145)


def cluster_snapshot(n_nodes, pods_per_node, n_its=400, seed=4205, n_pending=0, spot_frac=0.3, it_range=(15, 40),
                     uninitialized_frac=0.0, not_ready_frac=0.0, expire_after="720h", pod_selectors=False,
                     limits=None, topology=0, pdbs=False):
    """A consolidation snapshot: an existing cluster of `n_nodes` nodes launched from one
    WhenUnderutilized NodePool over fake.InstanceTypes(n_its), each running `pods_per_node` bound pods
    (C1 cpu/memory distributions, distinct pod-deletion-cost annotations so candidate costs are
    distinct), plus `n_pending` pending pods.  Every node is listed as a candidate; the host applies
    NewCandidate / filterCandidates / the disruption-cost sort.  Schema: INTEGRATION.md §5.

    topology=A > 0: the pods belong to A apps whose specs carry zonal / hostname spread (DoNotSchedule
    or ScheduleAnyway, some with minDomains), required hostname or zonal anti-affinity, or required /
    preferred zonal pod affinity; every bound pod is also listed in clusterPods (NewTopology's
    countDomains and inverse anti-affinity source).

    pdbs=True: PodDisruptionBudgets over the my-label values (some with no disruptions left, some with
    unhealthyPodEvictionPolicy AlwaysAllow) and some not-Ready pods (PDBLimits, pdblimits.go)."""
    rng = np.random.default_rng(seed)
    its = fake_instance_types(n_its)
    pool = node_pool("default", limits=limits)
    pool["spec"]["disruption"] = {"consolidationPolicy": "WhenUnderutilized", "expireAfter": expire_after}
    cpu_m = [100, 250, 500, 1000, 1500]
    mem_mi = [100, 256, 512, 1024, 2048, 4096]
    nodes, cands, cluster = [], [], []
    pid = 0
    apps = ["app-%d" % a for a in range(topology)]

    def app_spec(a):
        sel = {"matchLabels": {"app": apps[a]}}
        kind = a % 8
        if kind in (0, 1):
            c = {"maxSkew": 1 + a % 3, "topologyKey": ZONE, "labelSelector": sel,
                 "whenUnsatisfiable": "DoNotSchedule" if kind == 0 else "ScheduleAnyway"}
            if a % 5 == 0:
                c["minDomains"] = 3
            return {"topologySpreadConstraints": [c]}
        if kind in (2, 3):
            return {"topologySpreadConstraints": [{"maxSkew": 1 + a % 2, "topologyKey": HOSTNAME, "labelSelector": sel,
                                                   "whenUnsatisfiable": "DoNotSchedule" if kind == 2 else "ScheduleAnyway"}]}
        if kind == 4:
            return {"affinity": {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": sel, "topologyKey": HOSTNAME}]}}}
        if kind == 5:
            return {"affinity": {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": sel, "topologyKey": ZONE}]}}}
        if kind == 6:
            return {"affinity": {"podAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": 50, "podAffinityTerm": {"labelSelector": sel, "topologyKey": ZONE}}]}}}
        return {"affinity": {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": {"matchLabels": {"app": apps[(a + 1) % len(apps)]}}, "topologyKey": ZONE}]}}}

    for j in range(n_nodes):
        i = int(rng.integers(it_range[0], it_range[1]))
        it = its[i]
        alloc_cpu_m = (i + 1) * 1000 - 100
        alloc_mem = 2 * (i + 1) * GI - 10 * (1 << 20)
        alloc_pods = 10 * (i + 1)
        offers = [o for o in it["offerings"] if o["available"]]
        spot = rng.random() < spot_frac
        cands_off = [o for o in offers if o["capacityType"] == ("spot" if spot else "on-demand")]
        off = cands_off[int(rng.integers(len(cands_off)))]
        used_cpu, used_mem, pods = 0, 0, []
        for _ in range(pods_per_node):
            c = cpu_m[int(rng.integers(5))]
            m = mem_mi[int(rng.integers(6))] << 20
            if used_cpu + c > alloc_cpu_m or used_mem + m > alloc_mem or len(pods) + 1 > alloc_pods:
                continue
            used_cpu += c
            used_mem += m
            labels = {"my-label": LABEL_VALUES[rng.integers(7)]}
            a = int(rng.integers(topology)) if topology else -1
            if a >= 0:
                labels["app"] = apps[a]
            p = pod(pid, cpu="%dm" % c, mem="%dMi" % (m >> 20), labels=labels)
            if a >= 0:
                p["spec"].update(app_spec(a))
            if pod_selectors and rng.random() < 0.2:
                p["spec"]["nodeSelector"] = {ARCH: "amd64"}
            p["metadata"]["annotations"] = {"controller.kubernetes.io/pod-deletion-cost": str(int(rng.integers(-1000, 1000000)))}
            p["spec"]["nodeName"] = "node-%05d" % j
            p["status"] = {"phase": "Running", "conditions": [{"type": "PodScheduled", "status": "True"}]}
            if pdbs and rng.random() < 0.15:
                p["status"]["conditions"].append({"type": "Ready", "status": "False"})
            pods.append(p)
            if topology:
                cluster.append(p)
            pid += 1
        name = "node-%05d" % j
        labels = {NODEPOOL: "default", IT_LABEL: it["name"], ZONE: off["zone"], CT: off["capacityType"],
                  HOSTNAME: name, ARCH: "amd64", OS: "linux", "testing/cluster": "unspecified"}
        nodes.append({
            "name": name, "hostName": name, "labels": labels, "taints": [],
            "capacity": dict(it["capacity"]),
            "available": {"cpu": "%dm" % (alloc_cpu_m - used_cpu), "memory": str(alloc_mem - used_mem),
                          "pods": str(alloc_pods - len(pods))},
            "daemonSetRequests": {},
            "initialized": bool(rng.random() >= uninitialized_frac),
            "ready": bool(rng.random() >= not_ready_frac),
            "creationTimestamp": _fmt_time(NOW - int(rng.integers(0, 30 * 86400))),
            "pods": pods,
        })
        cands.append(name)
    pending = []
    for _ in range(n_pending):
        p = pod(pid, cpu=CPU_CHOICES[rng.integers(5)], mem=MEM_CHOICES[rng.integers(6)])
        if topology:
            a = int(rng.integers(topology))
            p["metadata"]["labels"]["app"] = apps[a]
            p["spec"].update(app_spec(a))
        pending.append(p)
        pid += 1
    return {
        "wellKnownLabels": FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": {"default": list(range(n_its))},
        "nodeClaimTemplates": [pool],
        "nodePools": [pool],
        "daemonSetPods": [],
        "stateNodes": nodes,
        "pendingPods": pending,
        "candidates": cands,
        "now": _fmt_time(NOW),
        "hostnameSeed": 0,
        **({"clusterPods": cluster} if topology else {}),
        **({"podDisruptionBudgets": _pdbs(rng)} if pdbs else {}),
    }


def _pdbs(rng):
    """Budgets over my-label: a (none left), b (none left, unhealthy pods always evictable), c|d (one
    left), e in another namespace (none left); f and g are unbudgeted."""
    z = int(rng.integers(0, 2))
    return [
        {"metadata": {"name": "pdb-a", "namespace": "default"}, "spec": {"selector": {"matchLabels": {"my-label": "a"}}},
         "status": {"disruptionsAllowed": 0}},
        {"metadata": {"name": "pdb-b", "namespace": "default"},
         "spec": {"selector": {"matchExpressions": [{"key": "my-label", "operator": "In", "values": ["b"]}]},
                  "unhealthyPodEvictionPolicy": "AlwaysAllow"}, "status": {"disruptionsAllowed": z}},
        {"metadata": {"name": "pdb-cd", "namespace": "default"},
         "spec": {"selector": {"matchExpressions": [{"key": "my-label", "operator": "In", "values": ["c", "d"]}]}},
         "status": {"disruptionsAllowed": 1}},
        {"metadata": {"name": "pdb-e", "namespace": "other"}, "spec": {"selector": {"matchLabels": {"my-label": "e"}}},
         "status": {"disruptionsAllowed": 0}},
    ]


def config5(n_nodes=5000, pods_per_node=20, seed=4205):
    """C5: multi-node + single-node consolidation over a 5k-node / 100k-pod cluster."""
    return cluster_snapshot(n_nodes, pods_per_node, 400, seed)


C3_ZONES = ["test-zone-1", "test-zone-2", "test-zone-3", "test-zone-4"]


def config4(n_pods=10000, n_nodes=2000, seed=4204, n_apps=20, limits=None, ghost_frac=0.0):
    """C4 (BASELINE.json configs[3]): pending pods with zonal + hostname topology spread and pod
    anti-affinity onto existing initialized nodes.  fake.InstanceTypes(400) offered in 4 zones x
    {spot, on-demand}; `n_nodes` nodes (8-32 cpu, unique hostnames, zones round-robin) 50-80 %
    utilised by bound cluster pods that carry the same app labels, so countDomains seeds every
    group.  `n_apps` apps as label selectors: the first half zonal spread maxSkew 1, the next 30 %
    hostname spread maxSkew 1, the rest required hostname anti-affinity.
    limits: NodePool limits (the pool is then also listed in nodePools); ghost_frac: that share of the
    pods carries required hostname pod affinity to an app no pod runs (unsatisfiable topology)."""
    rng = np.random.default_rng(seed)
    its = []
    for i in range(400):
        price = price_from_resources(i + 1, 2 * (i + 1) * GI)
        offers = [{"capacityType": ct, "zone": z, "price": price * (0.5 if ct == "spot" else 1.0), "available": True}
                  for z in C3_ZONES for ct in ("spot", "on-demand")]
        its.append(fake_instance_type("fake-it-%d" % i, i + 1, 2 * (i + 1), pods=10 * (i + 1), offerings=offers))
    pool = node_pool("default", limits=limits)
    apps = ["app-%02d" % a for a in range(n_apps)]
    n_zone, n_host = n_apps // 2, (n_apps * 3) // 10

    def app_spec(a):
        sel = {"matchLabels": {"app": apps[a]}}
        if a < n_zone:
            return {"topologySpreadConstraints": [{"maxSkew": 1, "topologyKey": ZONE, "whenUnsatisfiable": "DoNotSchedule",
                                                   "labelSelector": sel}]}
        if a < n_zone + n_host:
            return {"topologySpreadConstraints": [{"maxSkew": 1, "topologyKey": HOSTNAME,
                                                   "whenUnsatisfiable": "DoNotSchedule", "labelSelector": sel}]}
        return {"affinity": {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": sel, "topologyKey": HOSTNAME}]}}}

    cpu_m = [100, 250, 500, 1000, 1500]
    mem_mi = [100, 256, 512, 1024, 2048, 4096]
    nodes, cluster = [], []
    pid = 1000000
    for j in range(n_nodes):
        i = int(rng.integers(7, 32))
        alloc_cpu_m, alloc_mem, alloc_pods = (i + 1) * 1000 - 100, 2 * (i + 1) * GI - 10 * (1 << 20), 10 * (i + 1)
        target = float(rng.uniform(0.5, 0.8))
        used_cpu, used_mem, n_bound = 0, 0, 0
        name = "node-%05d" % j
        while used_cpu < target * alloc_cpu_m:
            c, m = cpu_m[int(rng.integers(5))], mem_mi[int(rng.integers(6))] << 20
            if used_cpu + c > alloc_cpu_m or used_mem + m > alloc_mem or n_bound + 1 >= alloc_pods:
                break
            a = int(rng.integers(n_apps))
            if a >= n_zone + n_host and any(cp["metadata"]["labels"]["app"] == apps[a] and
                                            cp["spec"]["nodeName"] == name for cp in cluster[-n_bound:] if n_bound):
                a = int(rng.integers(n_zone))  # keep the running anti-affinity pods one per host
            cp = pod(pid, cpu="%dm" % c, mem="%dMi" % (m >> 20), labels={"app": apps[a]})
            cp["spec"]["nodeName"] = name
            cp["status"] = {"phase": "Running"}
            cluster.append(cp)
            pid += 1
            used_cpu, used_mem, n_bound = used_cpu + c, used_mem + m, n_bound + 1
        zone = C3_ZONES[j % 4]
        ct = "spot" if rng.random() < 0.3 else "on-demand"
        labels = {NODEPOOL: "default", IT_LABEL: its[i]["name"], ZONE: zone, CT: ct, HOSTNAME: name, ARCH: "amd64",
                  OS: "linux", "testing/cluster": "unspecified"}
        nodes.append({
            "name": name, "hostName": name, "labels": labels, "taints": [],
            "capacity": dict(its[i]["capacity"]),
            "available": {"cpu": "%dm" % (alloc_cpu_m - used_cpu), "memory": str(alloc_mem - used_mem),
                          "pods": str(alloc_pods - n_bound)},
            "daemonSetRequests": {}, "initialized": True,
        })
    pods = []
    for i in range(n_pods):
        a = int(rng.integers(n_apps))
        p = pod(i, cpu=CPU_CHOICES[rng.integers(5)], mem=MEM_CHOICES[rng.integers(6)], labels={"app": apps[a]})
        p["spec"].update(app_spec(a))
        if ghost_frac and rng.random() < ghost_frac:
            p["spec"].pop("topologySpreadConstraints", None)
            p["spec"]["affinity"] = {"podAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchLabels": {"app": "ghost"}}, "topologyKey": HOSTNAME}]}}
        pods.append(p)
    return {
        "wellKnownLabels": FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": {"default": list(range(400))},
        "nodeClaimTemplates": [pool],
        "nodePools": [pool] if limits else [],
        "stateNodes": nodes,
        "daemonSetPods": [],
        "pods": pods,
        "clusterPods": cluster,
    }


def config3(n_pods=20000, seed=4203):
    """C3 (BASELINE.json configs[2]): pods with nodeSelector / required + preferred node affinity and
    tolerations over 800 instance types (100 cpu x memory shapes x 2 arch x 4 families), each offered
    in 4 zones x {spot, on-demand} (spot = 0.3 x the fake price), and 3 weighted NodePools with
    NoSchedule taints and zone / capacity-type requirements.  40 % of pods carry a nodeSelector
    (zone / arch / capacity-type), 30 % required node affinity (In / NotIn / Gt / Lt on `integer`),
    20 % preferred node affinity, 30 % tolerations."""
    rng = np.random.default_rng(seed)
    its = []
    shapes = [(c, m) for c in (1, 2, 4, 8, 16, 32, 48, 64, 96, 128) for m in (1, 2, 4, 6, 8, 12, 16, 24, 32, 48)][:100]
    for fam in ("c", "m", "r", "t"):
        for arch in ("amd64", "arm64"):
            for cpu, ratio in shapes:
                mem = cpu * ratio
                price = price_from_resources(cpu, mem * GI) * {"c": 1.0, "m": 1.1, "r": 1.3, "t": 0.9}[fam]
                offers = [{"capacityType": ct, "zone": z, "price": price * (0.3 if ct == "spot" else 1.0),
                           "available": bool(rng.random() < 0.95)}
                          for z in C3_ZONES for ct in ("spot", "on-demand")]
                name = "%s%d-%s-%dc-%dg" % (fam, len(its) % 7, arch, cpu, mem)
                its.append(fake_instance_type(name, cpu, mem, pods=min(250, 10 * cpu + 8), arch=arch,
                                              oses=("linux",), offerings=offers))
    pools = [
        node_pool("general", weight=10, requirements=[{"key": CT, "operator": "In", "values": ["on-demand", "spot"]}]),
        node_pool("spot-batch", weight=50, requirements=[{"key": CT, "operator": "In", "values": ["spot"]},
                                                          {"key": ZONE, "operator": "NotIn", "values": ["test-zone-4"]}],
                  taints=[{"key": "batch", "value": "true", "effect": "NoSchedule"}]),
        node_pool("gpu-team", weight=90, requirements=[{"key": ZONE, "operator": "In", "values": C3_ZONES[:2]}],
                  taints=[{"key": "team", "value": "ml", "effect": "NoSchedule"}], labels={"team": "ml"},
                  limits={"cpu": "20000"}),
    ]
    by_pool = {"general": list(range(len(its))), "spot-batch": [i for i in range(len(its)) if i % 2 == 0],
               "gpu-team": [i for i in range(len(its)) if its[i]["capacity"]["cpu"] not in ("1", "2")]}
    cpus, mems = CPU_CHOICES + ["2", "4"], MEM_CHOICES + ["8Gi"]
    pods = []
    for i in range(n_pods):
        p = pod(i, cpu=cpus[int(rng.integers(len(cpus)))], mem=mems[int(rng.integers(len(mems)))],
                labels={"my-label": LABEL_VALUES[int(rng.integers(7))]})
        spec = p["spec"]
        u = rng.random()
        if u < 0.4:
            k = int(rng.integers(3))
            spec["nodeSelector"] = [{ZONE: C3_ZONES[int(rng.integers(4))]},
                                    {ARCH: ("amd64", "arm64")[int(rng.integers(2))]},
                                    {CT: ("spot", "on-demand")[int(rng.integers(2))]}][k]
        elif u < 0.7:
            exprs = []
            v = int(rng.integers(4))
            if v == 0:
                exprs.append({"key": ZONE, "operator": "In", "values": sorted(set(
                    C3_ZONES[int(j)] for j in rng.integers(0, 4, size=2)))})
            elif v == 1:
                exprs.append({"key": ZONE, "operator": "NotIn", "values": [C3_ZONES[int(rng.integers(4))]]})
            elif v == 2:
                exprs.append({"key": "integer", "operator": "Gt", "values": [str(int(rng.choice([2, 4, 8, 16])))]})
            else:
                exprs.append({"key": "integer", "operator": "Lt", "values": [str(int(rng.choice([16, 32, 64])))]})
            terms = [{"matchExpressions": exprs}]
            if rng.random() < 0.3:
                terms.append({"matchExpressions": [{"key": ARCH, "operator": "In", "values": ["arm64"]}]})
            spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": terms}}}
        elif u < 0.9:
            spec["affinity"] = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [
                {"weight": int(rng.integers(1, 100)),
                 "preference": {"matchExpressions": [{"key": CT, "operator": "In", "values": ["spot"]}]}}]}}
        if rng.random() < 0.3:
            spec["tolerations"] = [[{"key": "batch", "operator": "Equal", "value": "true", "effect": "NoSchedule"}],
                                   [{"key": "team", "operator": "Exists"}],
                                   [{"operator": "Exists"}]][int(rng.integers(3))]
        pods.append(p)
    return {
        "wellKnownLabels": FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": by_pool,
        "nodeClaimTemplates": sorted(pools, key=lambda x: -x["spec"]["weight"]),
        "nodePools": pools,
        "stateNodes": [],
        "daemonSetPods": [],
        "pods": pods,
    }
