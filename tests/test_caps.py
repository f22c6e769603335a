"""Encoding caps past round 4's, GPU == oracle at about twice each old cap.

  NodePools      32 -> 64: a relaxation state's template-toleration set is one 64-bit mask (st_toltpl).
  taints        128 distinct -> 128 toleration classes: taints that exactly the same toleration lists tolerate
                share a mask bit (ks_host.cpp), so any number of distinct taints encodes while the pods' toleration
                lists tell at most 128 apart.
  host ports     64 triples -> 64 classes: (IP, port, protocol) entries that every pod being scheduled treats
                alike (conflict, reservation, own entry) share a bit; node entries no pod matches collapse.
  resources      16 names in any list -> 16 live names: the universe is the names the pods' / daemons' requests
                and the NodePool limits hold (Fits reads the candidate's names only, resources.go:162-175); an
                extra name's negative total still makes its instance type / node never fit.
The label-key universe stays at 64 referenced keys."""
import json

import pytest

import problems
from karpenter_amd import Scheduler, inspect
from oracle import bridge

CASES = [(k, s) for k in ("pools", "taints", "ports", "resources") for s in (1, 2, 3)]


def _names(snap, kind):
    if kind == "pools":
        return len(snap["nodeClaimTemplates"])
    if kind == "taints":
        ts = {(t["key"], t.get("value", ""), t["effect"]) for n in snap["stateNodes"] for t in n.get("taints", [])}
        ts |= {(t["key"], t.get("value", ""), t["effect"]) for p in snap["nodeClaimTemplates"]
               for t in p["spec"]["template"]["spec"].get("taints", [])}
        return len(ts)
    if kind == "ports":
        return len({(e["ip"], e["port"], e["protocol"]) for n in snap["stateNodes"]
                    for v in n.get("hostPortUsage", {}).values() for e in v})
    names = set()
    for it in snap["instanceTypes"]:
        names |= set(it["capacity"])
    return len(names)


@pytest.mark.parametrize("kind,seed", CASES, ids=["%s-%d" % c for c in CASES])
def test_caps_problem_encodes(kind, seed):
    snap = problems.caps_problem(seed, kind)
    old_cap = {"pools": 32, "taints": 128, "ports": 64, "resources": 16}[kind]
    assert _names(snap, kind) > old_cap * 1.7, _names(snap, kind)
    d = inspect(json.dumps(snap))
    if kind == "pools":
        assert d["templates"] == 64
    if kind == "resources":
        assert d["R"] <= 16
    res, _ = bridge.solve(json.dumps(snap))
    assert res["newNodeClaims"] or res["existingNodes"]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,seed", CASES, ids=["%s-%d" % c for c in CASES])
def test_caps_parity(kind, seed):
    snap = problems.caps_problem(seed, kind)
    s = json.dumps(snap)
    want, _ = bridge.solve(s)
    got = Scheduler(s).solve()
    assert got.canonical() == problems.canonical(want)
    if kind == "pools":  # templates past the 32nd are used
        names = {t["metadata"]["name"] for t in snap["nodeClaimTemplates"][32:]}
        assert any(c["nodePoolName"] in names for c in want["newNodeClaims"]), "no claim from a template past 32"
