"""Cluster-state deltas for ks_cons_update tests: apply one to a snapshot dict (what the cluster informers
would report after the events, state/cluster.go:220-512) and draw random ones.

apply_delta is written independently of the C++ update: it edits the snapshot JSON (pods move between
"pendingPods" and the nodes' "pods", StateNode "available" strings follow the pod requests, removed nodes
leave "stateNodes" and "candidates"; in a topology snapshot the "clusterPods" listing NewTopology counts
loses deleted pods and the removed nodes' pods and gains bound ones), and the oracle then consolidates the
edited snapshot from scratch.
"""
import copy
import random
from fractions import Fraction

_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": 1, "k": 10 ** 3,
        "M": 10 ** 6, "G": 10 ** 9, "T": 10 ** 12, "P": 10 ** 15, "E": 10 ** 18}


def parse_q(s):
    """resource.Quantity text -> exact value (the forms snapshots use: plain, decimal and binary suffixes)."""
    s = str(s)
    for suf, mul in _BIN.items():
        if s.endswith(suf):
            return Fraction(s[:-2]) * mul
    if s and s[-1] in _DEC and s[-1] != "" and not s[-1].isdigit():
        return Fraction(s[:-1]) * _DEC[s[-1]]
    return Fraction(s)


def fmt_q(v):
    if v.denominator == 1:
        return str(v.numerator)
    m = v * 1000
    if m.denominator == 1:
        return "%dm" % m.numerator
    n = v * 10 ** 9
    assert n.denominator == 1, v
    return "%dn" % n.numerator


def pod_requests(p):
    """RequestsForPods for the pods tests build (one or more containers with requests; pods = 1)."""
    spec = p["spec"]
    assert not spec.get("initContainers") and not spec.get("overhead"), "helper covers plain containers only"
    out = {"pods": Fraction(1)}
    for c in spec.get("containers", []):
        res = c.get("resources", {})
        assert not res.get("limits"), "helper covers requests only"
        for k, v in res.get("requests", {}).items():
            out[k] = out.get(k, Fraction(0)) + parse_q(v)
    return out


def _move(node, pod, sign):
    av = node["available"]
    for k, v in pod_requests(pod).items():
        if k in av:  # Subtract keeps the lhs keys only
            av[k] = fmt_q(parse_q(av[k]) + sign * v)


def _key(pod):
    return "%s/%s" % (pod["metadata"].get("namespace", "default"), pod["metadata"]["name"])


def _host_ports(pod):
    """GetHostPorts (hostportusage.go:92-114) as StateNode.HostPortUsage() reports them."""
    return [{"ip": e.get("hostIP", "0.0.0.0"), "port": e["hostPort"], "protocol": e.get("protocol", "TCP")}
            for c in pod["spec"].get("containers", []) for e in c.get("ports", []) if e.get("hostPort")]


def apply_delta(snap, delta):
    """The snapshot after ks_cons_update's delta (deletePods, then bindPods, then removeNodes)."""
    s = copy.deepcopy(snap)
    nodes = {n["name"]: n for n in s["stateNodes"]}
    listed = "clusterPods" in s

    def unlist(pred):
        if listed:
            s["clusterPods"] = [p for p in s["clusterPods"] if not pred(p)]

    for uid in delta.get("deletePods", []):
        unlist(lambda p: p["metadata"]["uid"] == uid)
        pend = [p for p in s.get("pendingPods", []) if p["metadata"]["uid"] == uid]
        if pend:
            s["pendingPods"].remove(pend[0])
            continue
        for n in s["stateNodes"]:
            hit = [p for p in n.get("pods", []) if p["metadata"]["uid"] == uid]
            if hit:
                n["pods"].remove(hit[0])
                _move(n, hit[0], +1)
                n.get("hostPortUsage", {}).pop(_key(hit[0]), None)  # HostPortUsage.DeletePod
                break
        else:
            raise KeyError(uid)
    for b in delta.get("bindPods", []):
        pod = [p for p in s["pendingPods"] if p["metadata"]["uid"] == b["uid"]][0]
        s["pendingPods"].remove(pod)
        pod["spec"]["nodeName"] = b["node"]
        pod["status"] = {"phase": "Running", "conditions": [{"type": "PodScheduled", "status": "True"}]}
        node = nodes[b["node"]]
        node.setdefault("pods", []).append(pod)
        _move(node, pod, -1)
        if _host_ports(pod):  # HostPortUsage.Add
            node.setdefault("hostPortUsage", {})[_key(pod)] = _host_ports(pod)
        unlist(lambda p: p["metadata"]["uid"] == b["uid"])
        if listed:
            s["clusterPods"].append(pod)
    for name in delta.get("removeNodes", []):
        unlist(lambda p: p.get("spec", {}).get("nodeName") == name)
        s["stateNodes"] = [n for n in s["stateNodes"] if n["name"] != name]
        s["candidates"] = [c for c in s.get("candidates", []) if c != name]
    return s


def random_delta(rng, snap, n_del=3, n_bind=2, n_rm=1):
    """A delta valid against `snap`: bound and pending pods deleted, pending pods bound to active nodes,
    nodes removed (with their pods)."""
    active = [n for n in snap["stateNodes"] if not n.get("markedForDeletion")]
    bound = [p["metadata"]["uid"] for n in active for p in n.get("pods", [])]
    pending = [p["metadata"]["uid"] for p in snap.get("pendingPods", [])]
    dels = rng.sample(bound, min(n_del, len(bound)))
    if pending and rng.random() < 0.5:
        dels.append(pending.pop(rng.randrange(len(pending))))
    binds = [{"uid": u, "node": rng.choice(active)["name"]} for u in rng.sample(pending, min(n_bind, len(pending)))]
    rms = [n["name"] for n in rng.sample(active, min(n_rm, len(active)))]
    return {"deletePods": dels, "bindPods": binds, "removeNodes": rms}


def delta_sequence(seed, snap, steps=4, **kw):
    """`steps` random deltas, each valid against the snapshot the previous ones lead to."""
    rng = random.Random(seed)
    out, cur = [], snap
    for _ in range(steps):
        d = random_delta(rng, cur, **kw)
        out.append(d)
        cur = apply_delta(cur, d)
    return out, cur
