"""Seeded random scheduling problems for oracle-vs-GPU parity tests.

Covers the Solve features the reference's suite_test.go / provisioning suite exercise: node
selectors, required node-affinity terms (In/NotIn/Exists/DoesNotExist/Gt/Lt, OR'd terms relaxed one
at a time), preferred node affinity (relaxed), tolerations vs NoSchedule / PreferNoSchedule taints,
NodePool limits, daemonset overhead, existing nodes (initialized / not), multiple weighted templates,
instance types with partial offerings.
"""
import numpy as np

from karpenter_amd import synth

ZONES = ["test-zone-1", "test-zone-2", "test-zone-3", "test-zone-4"]
CTS = ["spot", "on-demand"]
ARCHS = ["amd64", "arm64"]
TEAMS = ["red", "blue", "green"]


def _pick(rng, seq, k=None):
    if k is None:
        return seq[int(rng.integers(len(seq)))]
    idx = rng.choice(len(seq), size=min(k, len(seq)), replace=False)
    return [seq[int(i)] for i in sorted(idx)]


def random_its(rng, n):
    its = []
    for i in range(n):
        cpu = int(rng.choice([1, 2, 4, 8, 16, 32, 48, 64]))
        mem = int(cpu * rng.choice([1, 2, 4, 8]))
        offers = []
        for z in ZONES:
            for ct in CTS:
                if rng.random() < 0.45:
                    price = synth.price_from_resources(cpu, mem * synth.GI) * (0.3 if ct == "spot" else 1.0)
                    offers.append({"capacityType": ct, "zone": z, "price": price, "available": bool(rng.random() < 0.9)})
        if not offers:
            offers.append({"capacityType": "on-demand", "zone": ZONES[0], "price": 1.0, "available": True})
        it = synth.fake_instance_type("it-%03d-%dc%dg" % (i, cpu, mem), cpu, mem, pods=int(rng.choice([8, 16, 32, 110])),
                                      arch=_pick(rng, ARCHS), offerings=offers)
        if rng.random() < 0.1:
            it["capacity"]["example.com/gpu"] = str(int(rng.integers(1, 5)))
        its.append(it)
    return its


def random_nsr(rng, allow_custom=True):
    kind = rng.integers(7)
    if kind == 0:
        return {"key": synth.ZONE, "operator": "In", "values": _pick(rng, ZONES, int(rng.integers(1, 3)))}
    if kind == 1:
        return {"key": synth.ZONE, "operator": "NotIn", "values": _pick(rng, ZONES, 1)}
    if kind == 2:
        return {"key": synth.ARCH, "operator": "In", "values": [_pick(rng, ARCHS)]}
    if kind == 3:
        return {"key": synth.CT, "operator": "In", "values": [_pick(rng, CTS)]}
    if kind == 4:
        return {"key": "integer", "operator": _pick(rng, ["Gt", "Lt"]), "values": [str(int(rng.choice([2, 4, 8, 16, 32])))]}
    if kind == 5 and allow_custom:
        return {"key": "team", "operator": _pick(rng, ["In", "NotIn", "Exists", "DoesNotExist"]),
                "values": _pick(rng, TEAMS, 1)}
    return {"key": "size", "operator": _pick(rng, ["Exists", "DoesNotExist", "In"]), "values": ["large"]}


def random_pod(rng, i):
    cpu = _pick(rng, ["100m", "250m", "500m", "1", "1500m", "2", "3500m", "6"])
    mem = _pick(rng, ["128Mi", "512Mi", "1Gi", "1.8G", "3Gi", "6Gi", "12Gi"])
    p = synth.pod(i, cpu=cpu, mem=mem, labels={"app": "a%d" % (i % 5)})
    spec = p["spec"]
    if rng.random() < 0.25:
        sel = {}
        if rng.random() < 0.5:
            sel[synth.ZONE] = _pick(rng, ZONES)
        if rng.random() < 0.4:
            sel[synth.ARCH] = _pick(rng, ARCHS)
        if rng.random() < 0.2:
            sel["team"] = _pick(rng, TEAMS)
        if sel:
            spec["nodeSelector"] = sel
    aff = {}
    if rng.random() < 0.3:
        terms = [{"matchExpressions": [random_nsr(rng) for _ in range(int(rng.integers(1, 3)))]}
                 for _ in range(int(rng.integers(1, 4)))]
        aff.setdefault("nodeAffinity", {})["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": terms}
    if rng.random() < 0.2:
        prefs = [{"weight": int(rng.integers(1, 100)), "preference": {"matchExpressions": [random_nsr(rng)]}}
                 for _ in range(int(rng.integers(1, 3)))]
        aff.setdefault("nodeAffinity", {})["preferredDuringSchedulingIgnoredDuringExecution"] = prefs
    if aff:
        spec["affinity"] = aff
    if rng.random() < 0.3:
        tols = []
        if rng.random() < 0.6:
            tols.append({"key": "dedicated", "operator": "Equal", "value": _pick(rng, TEAMS), "effect": "NoSchedule"})
        if rng.random() < 0.3:
            tols.append({"operator": "Exists"})
        if rng.random() < 0.3:
            tols.append({"key": "spotty", "operator": "Exists"})
        if tols:
            spec["tolerations"] = tols
    if rng.random() < 0.05:
        spec["initContainers"] = [{"name": "init", "resources": {"requests": {"cpu": _pick(rng, ["2", "8", "100"])}}}]
    if rng.random() < 0.05:
        spec["containers"][0]["resources"]["requests"]["example.com/gpu"] = "1"
    return p


HOST_PORTS = [("", 80, "TCP"), ("", 443, "TCP"), ("10.0.0.1", 8080, "TCP"), ("0.0.0.0", 8080, "TCP"),
              ("10.0.0.2", 8080, "TCP"), ("", 53, "UDP"), ("::", 9090, "TCP"), ("fd00::1", 9090, "TCP")]


def add_host_ports(rng, pod):
    """hostPort container ports (hostportusage.go:92-114): IP / port / protocol combinations that do
    and do not Match each other (unspecified IPs match everything on the same port + protocol)."""
    ports = []
    for _ in range(int(rng.integers(1, 3))):
        ip, port, proto = HOST_PORTS[int(rng.integers(len(HOST_PORTS)))]
        e = {"containerPort": port, "hostPort": port, "protocol": proto}
        if ip:
            e["hostIP"] = ip
        ports.append(e)
    pod["spec"]["containers"][0]["ports"] = ports


VOL_DRIVERS = ["ebs.csi.aws.com", "fake.csi.provider", "efs.csi.aws.com", "unlimited.csi"]


def add_volumes(rng, pods, nodes):
    """PVC volumes (volumeusage.go:82-227): pods mount 0-3 of a 40-claim pool (persistentVolumeClaim or
    ephemeral <pod>-<volume>), claims resolve to one of 4 drivers, to "" (skipped) or not at all
    (NotFound, skipped); nodes carry CSINode limits for some drivers (0-6) and an existing usage that
    shares claims with the pods (sometimes already over its limit).  Returns the volumeDrivers map."""
    claims = ["claim-%02d" % i for i in range(40)]
    drivers = {}
    for c in claims:
        u = rng.random()
        if u < 0.85:
            drivers["default/" + c] = _pick(rng, VOL_DRIVERS)
        elif u < 0.92:
            drivers["default/" + c] = ""
    for p in pods:
        if rng.random() < 0.55:
            vols = []
            for k in range(int(rng.integers(1, 4))):
                if rng.random() < 0.15:
                    vols.append({"name": "eph%d" % k, "ephemeral": {"volumeClaimTemplate": {"spec": {}}}})
                    drivers["default/%s-eph%d" % (p["metadata"]["name"], k)] = _pick(rng, VOL_DRIVERS[:2])
                else:
                    vols.append({"name": "v%d" % k, "persistentVolumeClaim": {"claimName": _pick(rng, claims)}})
            p["spec"]["volumes"] = vols
    for n in nodes:
        lim = {}
        for d in VOL_DRIVERS[:3]:
            if rng.random() < 0.7:
                lim[d] = int(rng.integers(0, 7))
        usage = {}
        for d in VOL_DRIVERS:
            if rng.random() < 0.5:
                mine = ["default/bound-%s-%d" % (n["name"], i) for i in range(int(rng.integers(0, 3)))]
                shared = ["default/" + c for c in rng.choice(claims, size=int(rng.integers(0, 3)), replace=False)]
                usage[d] = sorted(set(mine + [c for c in shared if drivers.get(c) == d]))
        n["volumeLimits"] = lim
        n["volumeUsage"] = usage
    return drivers


OBJ_DRIVERS = ["ebs.csi.aws.com", "fake.csi.provider", "pd.csi.storage.gke.io", "disk.csi.azure.com",
               "efs.csi.aws.com", "d5.csi", "d6.csi", "unlimited.csi"]
IN_TREE = {"ebs.csi.aws.com": "kubernetes.io/aws-ebs", "pd.csi.storage.gke.io": "kubernetes.io/gce-pd",
           "disk.csi.azure.com": "kubernetes.io/azure-disk"}


def _resolve(claim, pvs, scs):
    """resolveDriver (volumeusage.go:119-155), for the generator's node usage lists only."""
    vn = claim["spec"].get("volumeName", "")
    if vn:
        pv = pvs.get(vn)
        if pv is None:
            return None
        src = pv["spec"]
        if src.get("csi"):
            return src["csi"]["driver"] or None
        if src.get("awsElasticBlockStore"):
            return "ebs.csi.aws.com"
    sc = scs.get(claim["spec"].get("storageClassName") or "")
    if sc is None:
        return None
    inv = {v: k for k, v in IN_TREE.items()}
    return inv.get(sc["provisioner"], sc["provisioner"])


def add_volume_objects(rng, pods, nodes, n_claims=300, share=0.1, zonal=0.5, broken=0.02, n_drivers=8,
                       own_usage=None, limit_range=(0, 8), mount_frac=0.6):
    """PersistentVolumeClaim / PersistentVolume / StorageClass objects instead of a volumeDrivers map: the
    library resolves drivers (resolveDriver, volumeusage.go:119-182, incl. the in-tree names of
    csi-translation-lib) and runs VolumeTopology.Inject (volumetopology.go:41-140) itself.  Pods mount 0-3
    claims, mostly their own (a StatefulSet's), a `share` fraction from a small pool (RWX); claims are bound to
    PVs (CSI, in-tree EBS or no CSI source, some with one or two zonal node-affinity terms) or unbound with a
    storage class (provisioner in-tree or CSI, zonal allowedTopologies or none, "" or missing); `broken` of the
    pods mount a missing claim or a claim bound to a missing PV (Inject fails; GetVolumes fails for the
    latter).  Nodes carry CSINode limits for most drivers and a usage list: `own_usage` maps node name ->
    pods bound there (their claims are mounted), plus some random claims.  Returns the three object lists."""
    drivers = OBJ_DRIVERS[:n_drivers]
    scs = {}
    for i, d in enumerate(drivers):
        for z in range(2):
            name = "sc-%d-%d" % (i, z)
            prov = IN_TREE[d] if d in IN_TREE and rng.random() < 0.5 else d
            sc = {"metadata": {"name": name}, "provisioner": prov}
            if z == 1 and rng.random() < zonal:
                zs = sorted(set(_pick(rng, ZONES) for _ in range(int(rng.integers(1, 3)))))
                sc["allowedTopologies"] = [{"matchLabelExpressions": [{"key": synth.ZONE, "values": zs}]}]
            scs[name] = sc
    pvs, pvcs = {}, {}

    def make_claim(ns, name):
        c = {"metadata": {"name": name, "namespace": ns}, "spec": {}}
        u = rng.random()
        if u < 0.5:
            pvname = "pv-%s-%s" % (ns, name)
            c["spec"]["volumeName"] = pvname
            c["spec"]["storageClassName"] = _pick(rng, sorted(scs)) if rng.random() < 0.7 else ""
            v = rng.random()
            spec = {}
            if v < 0.7:
                spec["csi"] = {"driver": _pick(rng, drivers), "volumeHandle": "h"}
            elif v < 0.85:
                spec["awsElasticBlockStore"] = {"volumeID": "vol-1", "fsType": "ext4"}
            if rng.random() < zonal:
                terms = [{"matchExpressions": [{"key": synth.ZONE, "operator": "In",
                                                "values": sorted(set(_pick(rng, ZONES) for _ in range(2)))}]}]
                if rng.random() < 0.2:
                    terms.append({"matchExpressions": [{"key": synth.ZONE, "operator": "In", "values": [_pick(rng, ZONES)]}]})
                spec["nodeAffinity"] = {"required": {"nodeSelectorTerms": terms}}
            pvs[pvname] = {"metadata": {"name": pvname}, "spec": spec}
        elif u < 0.96:
            c["spec"]["storageClassName"] = _pick(rng, sorted(scs))
        else:
            c["spec"]["storageClassName"] = ""
        pvcs[(ns, name)] = c
        return c

    pool = ["shared-%03d" % i for i in range(max(4, n_claims // 20))]
    next_claim = [0]

    def own(ns):
        next_claim[0] += 1
        return "claim-%05d" % next_claim[0]

    def anti_required(p):
        return bool(p["spec"].get("affinity", {}).get("podAntiAffinity", {}).get("requiredDuringSchedulingIgnoredDuringExecution"))

    for p in pods:
        ns = p["metadata"]["namespace"]
        if rng.random() >= mount_frac:
            continue
        vols = []
        for k in range(int(rng.integers(1, 4))):
            if rng.random() < 0.1:
                vols.append({"name": "eph%d" % k, "ephemeral": {"volumeClaimTemplate": {"spec": {}}}})
                make_claim(ns, "%s-eph%d" % (p["metadata"]["name"], k))
                continue
            name = _pick(rng, pool) if rng.random() < share else own(ns)
            if (ns, name) not in pvcs:
                make_claim(ns, name)
            vols.append({"name": "v%d" % k, "persistentVolumeClaim": {"claimName": name}})
        if rng.random() < broken and not anti_required(p):
            u = rng.random()
            if u < 0.3:
                vols.append({"name": "missing", "persistentVolumeClaim": {"claimName": "no-such-claim"}})
            elif u < 0.6:
                name = own(ns)
                pvcs[(ns, name)] = {"metadata": {"name": name, "namespace": ns},
                                    "spec": {"storageClassName": "missing-class"}}
                vols.append({"name": "noclass", "persistentVolumeClaim": {"claimName": name}})
            else:
                name = own(ns)
                pvcs[(ns, name)] = {"metadata": {"name": name, "namespace": ns}, "spec": {"volumeName": "no-such-pv"}}
                vols.append({"name": "gone", "persistentVolumeClaim": {"claimName": name}})
        p["spec"]["volumes"] = vols
    lo, hi = limit_range
    for n in nodes:
        lim = {d: int(rng.integers(lo, hi)) for d in drivers[:-1] if rng.random() < 0.8}
        usage = {}
        mounted = []
        for bp in (own_usage or {}).get(n["name"], []):
            for v in bp["spec"].get("volumes", []):
                name = v["persistentVolumeClaim"]["claimName"] if "persistentVolumeClaim" in v else \
                    "%s-%s" % (bp["metadata"]["name"], v["name"])
                mounted.append((bp["metadata"]["namespace"], name))
        keys = list(pvcs)
        for _ in range(int(rng.integers(0, 3))):
            if keys:
                mounted.append(keys[int(rng.integers(len(keys)))])
        for key in mounted:
            c = pvcs.get(key)
            if c is None:
                continue
            d = _resolve(c, pvs, scs)
            if d:
                usage.setdefault(d, set()).add("%s/%s" % key)
        for i in range(int(rng.integers(0, 3))):
            usage.setdefault(_pick(rng, drivers), set()).add("default/bound-%s-%d" % (n["name"], i))
        n["volumeLimits"] = lim
        n["volumeUsage"] = {d: sorted(v) for d, v in usage.items()}
    return list(pvcs.values()), list(pvs.values()), list(scs.values())


TOPO_KEYS = [synth.ZONE, synth.HOSTNAME, synth.CT]


def _app_selector(rng, app):
    if rng.random() < 0.8:
        return {"matchLabels": {"app": app}}
    return {"matchExpressions": [{"key": "app", "operator": _pick(rng, ["In", "NotIn"]),
                                  "values": sorted({app, "a%d" % int(rng.integers(5))})}]}


def _anti_term(rng, app):
    return {"labelSelector": _app_selector(rng, app), "topologyKey": _pick(rng, [synth.HOSTNAME, synth.HOSTNAME, synth.ZONE])}


def add_topology(rng, pods, nodes, affinity=False, or_terms=False):
    """Topology spread (zone / hostname / capacity-type, maxSkew 1-3, minDomains, DoNotSchedule and
    ScheduleAnyway), required + preferred pod anti-affinity (topology.go, topologygroup.go) per app,
    plus bound cluster pods on the existing nodes that seed the counts (countDomains) and inverse
    anti-affinity groups.  Pods carrying a spread constraint keep one required node-affinity term:
    relaxing OR'd terms would change the group's node filter mid-Solve (ks_topo.cpp refuses that)."""
    apps = {}
    for a in range(5):
        app = "a%d" % a
        spec = {}
        if rng.random() < 0.7:
            cs = []
            for key in _pick(rng, TOPO_KEYS, int(rng.integers(1, 3))):
                c = {"topologyKey": key, "maxSkew": int(rng.integers(1, 4)), "labelSelector": _app_selector(rng, app),
                     "whenUnsatisfiable": "ScheduleAnyway" if rng.random() < 0.25 else "DoNotSchedule"}
                if c["whenUnsatisfiable"] == "DoNotSchedule" and key != synth.HOSTNAME and rng.random() < 0.2:
                    c["minDomains"] = int(rng.integers(2, 5))
                cs.append(c)
            spec["tsc"] = cs
            f = rng.random()  # the app's node filter (nodeSelector / one required term), shared by its pods
            if f < 0.2:
                spec["sel"] = {synth.ZONE: _pick(rng, ZONES[:3])}
            elif f < 0.35:
                spec["sel"] = {synth.ARCH: _pick(rng, ARCHS)}
            elif f < 0.5:
                spec["req"] = [{"matchExpressions": [{"key": synth.ZONE, "operator": "In",
                                                      "values": sorted(_pick(rng, ZONES, 2))}]}]
            if or_terms and rng.random() < 0.7:  # OR'd terms: relaxing term[0] re-hashes the spread group
                spec.pop("sel", None)
                spec["req"] = [{"matchExpressions": [{"key": synth.ZONE, "operator": "In",
                                                      "values": sorted(_pick(rng, ZONES, int(rng.integers(1, 3))))}]}
                               for _ in range(int(rng.integers(2, 4)))]
        if rng.random() < 0.35:
            spec["anti"] = [_anti_term(rng, app)]
        if rng.random() < 0.25:
            spec["antiPref"] = [{"weight": int(rng.integers(1, 100)), "podAffinityTerm": _anti_term(rng, app)}]
        if affinity and rng.random() < 0.3:  # to itself or to another app, zone or hostname
            other = app if rng.random() < 0.5 else "a%d" % int(rng.integers(5))
            spec["aff"] = [{"labelSelector": {"matchLabels": {"app": other}},
                            "topologyKey": _pick(rng, [synth.ZONE, synth.HOSTNAME, synth.CT])}]
        if affinity and rng.random() < 0.2:
            spec["affPref"] = [{"weight": int(rng.integers(1, 100)), "podAffinityTerm": {
                "labelSelector": {"matchLabels": {"app": "a%d" % int(rng.integers(5))}},
                "topologyKey": _pick(rng, [synth.ZONE, synth.HOSTNAME])}}]
        apps[app] = spec
    for p in pods:
        app = p["metadata"]["labels"]["app"]
        spec = apps[app]
        if rng.random() < 0.15:
            continue  # some pods of the app carry no constraint (still counted by the selectors)
        if "tsc" in spec:
            p["spec"]["topologySpreadConstraints"] = spec["tsc"]
            p["spec"].pop("nodeSelector", None)
            if "sel" in spec:
                p["spec"]["nodeSelector"] = dict(spec["sel"])
            na = p["spec"].get("affinity", {}).get("nodeAffinity", {})
            na.pop("requiredDuringSchedulingIgnoredDuringExecution", None)
            if "req" in spec:
                na = p["spec"].setdefault("affinity", {}).setdefault("nodeAffinity", {})
                na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": spec["req"]}
            elif "affinity" in p["spec"] and p["spec"]["affinity"].get("nodeAffinity") == {}:
                del p["spec"]["affinity"]["nodeAffinity"]
        if "anti" in spec or "antiPref" in spec:
            paa = {}
            if "anti" in spec:
                paa["requiredDuringSchedulingIgnoredDuringExecution"] = spec["anti"]
            if "antiPref" in spec:
                paa["preferredDuringSchedulingIgnoredDuringExecution"] = spec["antiPref"]
            p["spec"].setdefault("affinity", {})["podAntiAffinity"] = paa
        if "aff" in spec or "affPref" in spec:
            pa = {}
            if "aff" in spec:
                pa["requiredDuringSchedulingIgnoredDuringExecution"] = spec["aff"]
            if "affPref" in spec:
                pa["preferredDuringSchedulingIgnoredDuringExecution"] = spec["affPref"]
            p["spec"].setdefault("affinity", {})["podAffinity"] = pa
    cluster = []
    for i, n in enumerate(nodes):
        for j in range(int(rng.integers(0, 4))):
            app = "a%d" % int(rng.integers(5))
            cp = synth.pod(500000 + i * 10 + j, cpu="100m", labels={"app": app})
            cp["spec"]["nodeName"] = n["name"]
            cp["status"] = {"phase": _pick(rng, ["Running", "Running", "Running", "Succeeded"])}
            if rng.random() < 0.15:
                cp["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                    {"labelSelector": {"matchLabels": {"app": "a%d" % int(rng.integers(5))}},
                     "topologyKey": _pick(rng, [synth.HOSTNAME, synth.ZONE])}]}}
            cluster.append(cp)
    return cluster


NAMESPACES = [("default", {"env": "prod"}), ("team-a", {"env": "prod", "team": "a"}), ("team-b", {"env": "dev"}),
              ("kube-system", {})]


def add_namespaces(rng, pods, cluster):
    """Spread pods and cluster pods over four namespaces and give the (anti-)affinity terms a
    namespace list or a namespaceSelector (buildNamespaceList, topology.go:339-362): empty (every
    namespace), by label, or matching nothing.  Returns the snapshot's namespace list."""
    terms = []
    for p in pods + cluster:
        p["metadata"]["namespace"] = _pick(rng, [n for n, _ in NAMESPACES[:3]])
        aff = p["spec"].get("affinity", {})
        for kind in ("podAffinity", "podAntiAffinity"):
            for t in aff.get(kind, {}).get("requiredDuringSchedulingIgnoredDuringExecution", []):
                terms.append(t)
            for w in aff.get(kind, {}).get("preferredDuringSchedulingIgnoredDuringExecution", []):
                terms.append(w["podAffinityTerm"])
    seen = set()
    for t in terms:  # app specs share term dicts: decide once per dict
        if id(t) in seen:
            continue
        seen.add(id(t))
        u = rng.random()
        if u < 0.2:
            t["namespaceSelector"] = {}
        elif u < 0.4:
            t["namespaceSelector"] = {"matchLabels": {"env": _pick(rng, ["prod", "dev"])}}
        elif u < 0.5:
            t["namespaceSelector"] = {"matchExpressions": [{"key": "team", "operator": "Exists"}]}
            t["namespaces"] = ["team-b"]
        elif u < 0.6:
            t["namespaces"] = ["default", "team-a"]
    return [{"name": n, "labels": lab} for n, lab in NAMESPACES]


def special_nsr(rng):
    """A term on the fake instance types' 'special' key, the one key some instance types hold as
    DoesNotExist (fake/instancetype.go: small types): Exists + NotIn is NotIn, which a DoesNotExist
    instance type intersects (requirements.go:248-252), so the factorised feasibility rows must not
    decide those positions from one side alone."""
    op = _pick(rng, ["In", "NotIn", "NotIn", "Exists", "Exists", "DoesNotExist"])
    e = {"key": "special", "operator": op}
    if op in ("In", "NotIn"):
        e["values"] = ["optional"]
    return e


def random_problem(seed, n_pods=120, n_its=40, n_nodes=None, n_templates=None, host_ports=False, topology=False,
                   affinity=False, volumes=False, namespaces=False, same_pod_ports=False, or_terms=False,
                   special=False, volume_objects=None):
    """same_pod_ports: existing nodes' HostPortUsage also holds entries keyed by pods being scheduled
    (their own ports, or others), the case HostPortUsage.Conflicts skips and Add replaces
    (hostportusage.go:70-85).  special: NodePool and pod terms on the 'special' key (special_nsr)."""
    rng = np.random.default_rng(seed)
    its = random_its(rng, n_its)
    n_templates = int(rng.integers(1, 4)) if n_templates is None else n_templates
    templates, pools, by_pool = [], [], {}
    for t in range(n_templates):
        name = "pool-%d" % t
        reqs = [random_nsr(rng, allow_custom=False) for _ in range(int(rng.integers(0, 2)))]
        if special and rng.random() < 0.7:
            reqs.append(special_nsr(rng))
        taints = []
        if rng.random() < 0.35:
            taints.append({"key": "dedicated", "value": _pick(rng, TEAMS), "effect": "NoSchedule"})
        if rng.random() < 0.2:
            taints.append({"key": "spotty", "value": "", "effect": "PreferNoSchedule"})
        labels = {"team": _pick(rng, TEAMS)} if rng.random() < 0.5 else {}
        limits = {"cpu": str(int(rng.choice([16, 64, 256, 1000])))} if rng.random() < 0.4 else None
        np_obj = synth.node_pool(name, weight=int(rng.integers(0, 100)), limits=limits, requirements=reqs,
                                 taints=taints, labels=labels)
        templates.append(np_obj)
        pools.append(np_obj)
        k = max(1, int(n_its * rng.uniform(0.3, 1.0)))
        by_pool[name] = sorted(int(i) for i in rng.choice(n_its, size=k, replace=False))
    # Provisioner.NewScheduler orders templates by weight (nodepool.go:209-213); keep that order.
    order = sorted(range(n_templates), key=lambda i: -templates[i]["spec"].get("weight", 0))
    templates = [templates[i] for i in order]
    n_nodes = int(rng.integers(0, 12)) if n_nodes is None else n_nodes
    nodes = []
    for i in range(n_nodes):
        pool = templates[int(rng.integers(len(templates)))]["metadata"]["name"]
        cpu = int(rng.choice([2, 4, 8, 16]))
        name = "node-%03d" % i
        labels = {synth.ZONE: _pick(rng, ZONES), synth.ARCH: _pick(rng, ARCHS), synth.NODEPOOL: pool,
                  synth.HOSTNAME: name, synth.CT: _pick(rng, CTS)}
        if rng.random() < 0.5:
            labels["team"] = _pick(rng, TEAMS)
        taints = [{"key": "dedicated", "value": _pick(rng, TEAMS), "effect": "NoSchedule"}] if rng.random() < 0.2 else []
        used = float(rng.uniform(0, 0.8))
        nodes.append({
            "name": name, "hostName": name, "labels": labels, "taints": taints,
            "available": {"cpu": "%dm" % int(cpu * 1000 * (1 - used)), "memory": "%dMi" % int(cpu * 2048 * (1 - used)),
                          "pods": str(int(rng.integers(0, 30)))},
            "capacity": {"cpu": str(cpu), "memory": "%dGi" % (cpu * 2), "pods": "110"},
            "daemonSetRequests": {"cpu": "100m"} if rng.random() < 0.5 else {},
            "initialized": bool(rng.random() < 0.8),
        })
        if host_ports and rng.random() < 0.5:
            ip, port, proto = HOST_PORTS[int(rng.integers(len(HOST_PORTS)))]
            nodes[-1]["hostPortUsage"] = {"default/bound-%d" % i: [{"ip": ip or "0.0.0.0", "port": port,
                                                                   "protocol": proto}]}
    daemons = []
    for i in range(int(rng.integers(0, 3))):
        d = synth.pod(100000 + i, cpu=_pick(rng, ["50m", "100m", "200m"]), mem=_pick(rng, ["64Mi", "128Mi"]))
        if rng.random() < 0.5:
            d["spec"]["tolerations"] = [{"operator": "Exists"}]
        if rng.random() < 0.3:
            d["spec"]["nodeSelector"] = {synth.ARCH: _pick(rng, ARCHS)}
        daemons.append(d)
    pods = [random_pod(rng, i) for i in range(n_pods)]
    if special:
        for p in pods:
            if rng.random() < 0.45:
                e = special_nsr(rng)
                na = p["spec"].setdefault("affinity", {}).setdefault("nodeAffinity", {})
                req = na.setdefault("requiredDuringSchedulingIgnoredDuringExecution",
                                    {"nodeSelectorTerms": [{"matchExpressions": []}]})
                for term in req["nodeSelectorTerms"]:
                    term.setdefault("matchExpressions", []).append(dict(e))
    if host_ports:
        for p in pods:
            if rng.random() < 0.4:
                add_host_ports(rng, p)
    if same_pod_ports and nodes:
        for p in pods:
            if rng.random() < 0.1:
                n = nodes[int(rng.integers(len(nodes)))]
                own = p["spec"]["containers"][0].get("ports") or []
                if own and rng.random() < 0.7:
                    entries = [{"ip": e.get("hostIP", "0.0.0.0"), "port": e["hostPort"], "protocol": e["protocol"]}
                               for e in own]
                else:
                    ip, port, proto = HOST_PORTS[int(rng.integers(len(HOST_PORTS)))]
                    entries = [{"ip": ip or "0.0.0.0", "port": port, "protocol": proto}]
                n.setdefault("hostPortUsage", {})["%s/%s" % (p["metadata"]["namespace"], p["metadata"]["name"])] = entries
    cluster = add_topology(rng, pods, nodes, affinity, or_terms) if topology else []
    nss = add_namespaces(rng, pods, cluster) if namespaces else []
    vdrivers = add_volumes(rng, pods, nodes) if volumes else {}
    vobj = {}
    if volume_objects is not None:  # dict of add_volume_objects keyword arguments
        pvcs, pvs, scs = add_volume_objects(rng, pods, nodes, **volume_objects)
        vobj = {"persistentVolumeClaims": pvcs, "persistentVolumes": pvs, "storageClasses": scs}
    return {
        **({"namespaces": nss} if namespaces else {}),
        **({"volumeDrivers": vdrivers} if volume_objects is None else vobj),
        "wellKnownLabels": synth.FAKE_WELL_KNOWN,
        "instanceTypes": its,
        "instanceTypesByNodePool": by_pool,
        "nodeClaimTemplates": templates,
        "nodePools": pools,
        "stateNodes": nodes,
        "daemonSetPods": daemons,
        "pods": pods,
        "clusterPods": cluster,
    }


def hostname_failure_problem(seed, n_pods=150, n_nodes=8):
    """Pods whose hostname-keyed pod affinity no domain can satisfy, so Topology.AddRequirements fails
    with "unsatisfiable topology constraint ... (counts = map[...])" and prints every registered
    hostname domain with its count (topology.go:167): existing nodes (NewExistingNode registers them),
    every hostname-placeholder NewNodeClaim registered so far, and the counts this Solve recorded.
    Kinds: affinity to an app no pod carries ("ghost"), and affinity to an app that runs on the existing
    nodes while a hostname NotIn excludes every existing node (the target's pods then sit only on
    excluded domains until one lands on a NodeClaim)."""
    snap = random_problem(seed, n_pods=n_pods, n_nodes=n_nodes, topology=True, affinity=True)
    rng = np.random.default_rng(seed + 7919)
    names = [n["name"] for n in snap["stateNodes"]]
    for p in snap["pods"]:
        u = rng.random()
        if u >= 0.35:
            continue
        aff = p["spec"].setdefault("affinity", {})
        if u < 0.15:
            target = "ghost"
        else:
            target = "a%d" % int(rng.integers(5))
            if p["metadata"]["labels"]["app"] == target:
                continue
            na = aff.setdefault("nodeAffinity", {})
            na["requiredDuringSchedulingIgnoredDuringExecution"] = {"nodeSelectorTerms": [{"matchExpressions": [
                {"key": synth.HOSTNAME, "operator": "NotIn", "values": list(names) or ["nowhere"]}]}]}
        aff["podAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": [
            {"labelSelector": {"matchLabels": {"app": target}}, "topologyKey": synth.HOSTNAME}]}
        p["spec"].pop("topologySpreadConstraints", None)
    return snap


def canonical(results):
    d = dict(results)
    d.pop("stats", None)
    return d


def unlabel_topology_nodes(snap, seed, frac=0.3):
    """Existing nodes without the zone / capacity-type label a topology group keys on, and pods that
    admit them through a NotIn (or DoesNotExist) requirement on that key: ExistingNode.Add then takes
    the key from the pod's requirements and picks the domain like a NodeClaim's (existingnode.go:91-115)."""
    rng = np.random.default_rng(seed)
    for n in snap["stateNodes"]:
        if rng.random() < frac:
            for key in (synth.ZONE, synth.CT):
                if rng.random() < 0.6:
                    n["labels"].pop(key, None)
    for p in snap["pods"]:
        if rng.random() >= 0.35:
            continue
        key = synth.ZONE if rng.random() < 0.7 else synth.CT
        op = "NotIn" if rng.random() < 0.85 else "DoesNotExist"
        expr = {"key": key, "operator": op}
        if op == "NotIn":
            expr["values"] = sorted(_pick(rng, ZONES if key == synth.ZONE else CTS, 1))
        na = p["spec"].setdefault("affinity", {}).setdefault("nodeAffinity", {})
        req = na.setdefault("requiredDuringSchedulingIgnoredDuringExecution", {"nodeSelectorTerms": [{"matchExpressions": []}]})
        for term in req["nodeSelectorTerms"]:
            term.setdefault("matchExpressions", []).append(dict(expr))
    return snap


def many_groups_problem(seed, n_apps=150, n_pods=600, n_nodes=30, n_its=40):
    """A Solve whose topology has far more than 64 groups (one spread or anti-affinity group
    per deployment is what production clusters carry): n_apps apps, each with its own zonal or hostname
    spread (DoNotSchedule or ScheduleAnyway, maxSkew 1-3, some minDomains), some with required or preferred
    hostname / zonal anti-affinity or pod affinity to another app; bound cluster pods of every app on the
    existing nodes seed the counts, and some of them carry required anti-affinity (inverse groups)."""
    rng = np.random.default_rng(seed)
    snap = random_problem(seed, n_pods=n_pods, n_its=n_its, n_nodes=n_nodes)
    apps = {}
    for a in range(n_apps):
        app = "m%d" % a
        spec = {}
        if rng.random() < 0.8:
            key = _pick(rng, [synth.ZONE, synth.HOSTNAME, synth.ZONE, synth.CT])
            c = {"topologyKey": key, "maxSkew": int(rng.integers(1, 4)), "labelSelector": {"matchLabels": {"app": app}},
                 "whenUnsatisfiable": "ScheduleAnyway" if rng.random() < 0.2 else "DoNotSchedule"}
            if c["whenUnsatisfiable"] == "DoNotSchedule" and key != synth.HOSTNAME and rng.random() < 0.15:
                c["minDomains"] = int(rng.integers(2, 4))
            spec["tsc"] = [c]
        if rng.random() < 0.3:
            spec["anti"] = [{"labelSelector": {"matchLabels": {"app": app}},
                             "topologyKey": _pick(rng, [synth.HOSTNAME, synth.ZONE])}]
        elif rng.random() < 0.2:
            spec["antiPref"] = [{"weight": int(rng.integers(1, 100)), "podAffinityTerm": {
                "labelSelector": {"matchLabels": {"app": app}}, "topologyKey": synth.HOSTNAME}}]
        if rng.random() < 0.1:
            spec["aff"] = [{"labelSelector": {"matchLabels": {"app": "m%d" % int(rng.integers(n_apps))}},
                            "topologyKey": synth.ZONE}]
        apps[app] = spec
    for i, p in enumerate(snap["pods"]):
        app = "m%d" % (i % n_apps)
        p["metadata"]["labels"]["app"] = app
        sp = p["spec"]
        sp.pop("nodeSelector", None)
        sp.pop("affinity", None)
        spec = apps[app]
        if "tsc" in spec:
            sp["topologySpreadConstraints"] = spec["tsc"]
        aff = {}
        if "anti" in spec:
            aff["podAntiAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": spec["anti"]}
        if "antiPref" in spec:
            aff["podAntiAffinity"] = {"preferredDuringSchedulingIgnoredDuringExecution": spec["antiPref"]}
        if "aff" in spec:
            aff["podAffinity"] = {"requiredDuringSchedulingIgnoredDuringExecution": spec["aff"]}
        if aff:
            sp["affinity"] = aff
    cluster = []
    for j, n in enumerate(snap["stateNodes"]):
        for k in range(int(rng.integers(0, 5))):
            app = "m%d" % int(rng.integers(n_apps))
            cp = synth.pod(200000 + 10 * j + k, cpu="100m", mem="64Mi", labels={"app": app})
            cp["metadata"]["name"] = "bound-%d-%d" % (j, k)
            cp["spec"]["nodeName"] = n["name"]
            cp["status"] = {"phase": "Running"}
            if rng.random() < 0.15:
                cp["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                    {"labelSelector": {"matchLabels": {"app": "m%d" % int(rng.integers(n_apps))}},
                     "topologyKey": _pick(rng, [synth.HOSTNAME, synth.ZONE])}]}}
            cluster.append(cp)
    snap["clusterPods"] = cluster
    return snap


def caps_problem(seed, kind, n_pods=300):
    """A random problem past one of the round-4 encoding caps, at about twice the cap:

    pools:     64 NodePools (templates), most tainted with a key of their own that few pods tolerate, so the
               pods spread over templates past the 32nd (st_toltpl is one 64-bit mask);
    taints:    ~280 distinct taints (40 keys x 7 values) on nodes and templates, tolerated by key (Exists) or by
               one value (Equal): more than 128 taints, at most ~90 toleration classes (ks_host.cpp);
    ports:     ~140 distinct (IP, port, protocol) entries in the nodes' HostPortUsage, the pods' ports a
               20-port subset that overlaps them: more than 64 triples, few classes;
    resources: ~34 resource names in the instance types' and nodes' capacity (and a node whose extra resource is
               overcommitted, an instance type whose overhead exceeds an extra resource), the pods requesting
               cpu / memory and a few extended names, NodePool limits on one: more than 16 names, fewer live."""
    rng = np.random.default_rng(seed)
    if kind == "pools":
        snap = random_problem(seed, n_pods=n_pods, n_templates=64, n_nodes=int(rng.integers(4, 12)))
        for t, tpl in enumerate(snap["nodeClaimTemplates"]):
            if t < 56:
                tpl["spec"]["template"]["spec"]["taints"] = [{"key": "pool-only-%d" % t, "value": "x",
                                                              "effect": "NoSchedule"}]
        for p in snap["pods"]:
            tols = p["spec"].setdefault("tolerations", [])
            for t in rng.choice(64, size=int(rng.integers(0, 4)), replace=False):
                tols.append({"key": "pool-only-%d" % int(t), "operator": "Exists"})
            if not tols:
                p["spec"].pop("tolerations")
        return snap
    snap = random_problem(seed, n_pods=n_pods, n_nodes=int(rng.integers(20, 40)), host_ports=(kind == "ports"))
    if kind == "taints":
        keys = ["taint-key-%02d" % k for k in range(40)]
        vals = ["v%d" % v for v in range(7)]
        for n in snap["stateNodes"]:
            n["taints"] = [{"key": keys[int(rng.integers(40))], "value": vals[int(rng.integers(7))],
                            "effect": _pick(rng, ["NoSchedule", "NoExecute"])} for _ in range(int(rng.integers(0, 4)))]
        all_taints = [{"key": k, "value": v, "effect": "NoSchedule"} for k in keys for v in vals]
        for i, tpl in enumerate(snap["nodeClaimTemplates"]):
            picks = rng.choice(len(all_taints), size=int(rng.integers(0, 3)), replace=False)
            tpl["spec"]["template"]["spec"]["taints"] = [all_taints[int(j)] for j in picks]
        # every (key, value) pair appears somewhere: 280 distinct taints
        extra = {"name": "taint-carrier", "hostName": "taint-carrier",
                 "labels": dict(snap["stateNodes"][0]["labels"], **{synth.HOSTNAME: "taint-carrier"}),
                 "taints": all_taints, "available": {"cpu": "4", "memory": "8Gi", "pods": "20"},
                 "capacity": {"cpu": "4", "memory": "8Gi", "pods": "110"}, "daemonSetRequests": {}, "initialized": True}
        snap["stateNodes"].append(extra)
        for p in snap["pods"]:
            if rng.random() < 0.6:
                tols = []
                for k in rng.choice(40, size=int(rng.integers(1, 12)), replace=False):
                    if rng.random() < 0.7:
                        tols.append({"key": keys[int(k)], "operator": "Exists"})
                    else:
                        tols.append({"key": keys[int(k)], "operator": "Equal", "value": "v0"})
                p["spec"]["tolerations"] = tols
        return snap
    if kind == "ports":
        ports = [("", 30000 + i, "TCP") for i in range(60)] + [("10.0.%d.1" % (i % 4), 31000 + i, "TCP") for i in range(50)] + \
                [("", 32000 + i, "UDP") for i in range(40)]
        for i, n in enumerate(snap["stateNodes"]):
            use = n.setdefault("hostPortUsage", {})
            for j in range(int(rng.integers(2, 8))):
                ip, port, proto = ports[int(rng.integers(len(ports)))]
                use["default/bound-%d-%d" % (i, j)] = [{"ip": ip or "0.0.0.0", "port": port, "protocol": proto}]
        if snap["stateNodes"]:  # every entry on some node: 150 distinct triples
            snap["stateNodes"][0]["hostPortUsage"]["default/port-carrier"] = [
                {"ip": ip or "0.0.0.0", "port": port, "protocol": proto} for ip, port, proto in ports]
        hot = [ports[int(i)] for i in rng.choice(len(ports), size=20, replace=False)]
        for p in snap["pods"]:
            if rng.random() < 0.3:
                e = []
                for _ in range(int(rng.integers(1, 3))):
                    ip, port, proto = hot[int(rng.integers(len(hot)))]
                    x = {"containerPort": port, "hostPort": port, "protocol": proto}
                    if ip:
                        x["hostIP"] = ip
                    e.append(x)
                p["spec"]["containers"][0]["ports"] = e
        return snap
    assert kind == "resources", kind
    names = ["example.com/res-%02d" % k for k in range(30)]
    for it in snap["instanceTypes"]:
        for k in rng.choice(30, size=int(rng.integers(10, 30)), replace=False):
            it["capacity"][names[int(k)]] = str(int(rng.integers(1, 9)))
    it = snap["instanceTypes"][int(rng.integers(len(snap["instanceTypes"])))]
    it["capacity"][names[29]] = "1"
    it["overhead"]["kubeReserved"][names[29]] = "2"  # allocatable -1 of a name no pod requests: never fits
    for n in snap["stateNodes"]:
        for k in rng.choice(30, size=int(rng.integers(5, 30)), replace=False):
            n["capacity"][names[int(k)]] = "8"
            n["available"][names[int(k)]] = str(int(rng.integers(0, 9)))
    if snap["stateNodes"]:
        snap["stateNodes"][0]["available"][names[28]] = "-1"  # overcommitted, not requested: never fits
    for p in snap["pods"]:
        if rng.random() < 0.3:
            req = p["spec"]["containers"][0]["resources"]["requests"]
            for k in rng.choice(6, size=int(rng.integers(1, 3)), replace=False):
                req[names[int(k)]] = str(int(rng.integers(1, 3)))
    pool = snap["nodeClaimTemplates"][0]
    pool["spec"].setdefault("limits", {})[names[7]] = "1000"
    for np_obj in snap["nodePools"]:
        if np_obj["metadata"]["name"] == pool["metadata"]["name"]:
            np_obj["spec"]["limits"] = dict(pool["spec"]["limits"])
    return snap
