"""Diagnose a consolidation simulation that differs from the oracle: rebuild it as a plain Solve snapshot
(helpers.go:73-127: the active nodes minus the candidates, pending + the candidates' pods + the deleting nodes'
pods) and compare GPU Solve vs oracle Solve vs the simulation records.  Profiling / debugging aid, not a test.
Usage: python scripts/cons_sim_diag.py <seed> [topology 0/1]"""
import copy
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "karpenter-sigs_amd"))

from oracle import bridge  # noqa: E402
import carry_scenarios as cs  # noqa: E402


def node_pods(n):  # GetNodePods (node.go:32-53), as the snapshot's pods carry it
    return [p for p in n.get("pods", []) if not p.get("metadata", {}).get("deletionTimestamp")]


def as_solve(snap, cand_names):
    s = copy.deepcopy(snap)
    nodes = s["stateNodes"]
    cset = set(cand_names)
    pods = list(s.get("pendingPods", []))
    for name in cand_names:
        n = next(x for x in nodes if x["name"] == name)
        pods += node_pods(n)
    for n in nodes:
        if n.get("markedForDeletion"):
            pods += node_pods(n)
    s["stateNodes"] = [n for n in nodes if n["name"] not in cset and not n.get("markedForDeletion")]
    s["pods"] = pods
    for k in ("pendingPods", "candidates", "now"):
        s.pop(k, None)
    return s


def main():
    seed = int(sys.argv[1])
    topo = len(sys.argv) < 3 or sys.argv[2] == "1"
    snap = cs.random_cluster(seed, topology=topo)
    from karpenter_amd import Consolidator, Scheduler
    want, _ = bridge.consolidate(json.dumps(snap), all_sims=True)
    res = {}
    for mode in ("tact", "notact"):
        if mode == "notact":
            os.environ["KS_NO_TACT"] = "1"
        else:
            os.environ.pop("KS_NO_TACT", None)
        got = Consolidator(json.dumps(snap)).consolidate(all_sims=True)
        got.pop("kernel_ms")
        res[mode] = got
    os.environ.pop("KS_NO_TACT", None)
    for method in ("multi", "single"):
        for i, (w, g, g2) in enumerate(zip(want[method]["sims"], res["tact"][method]["sims"], res["notact"][method]["sims"])):
            if w == g and w == g2:
                continue
            print("%s sim %d %s: oracle==tact %s oracle==notact %s" % (method, i, w["candidates"], w == g, w == g2))
            ss = as_solve(snap, w["candidates"])
            o, _ = bridge.solve(json.dumps(ss))
            gs = Scheduler(json.dumps(ss)).solve().canonical()
            o.pop("stats", None)
            gs.pop("stats", None)
            print("   solve GPU == oracle:", gs == o)
            if o["newNodeClaims"]:
                print("   oracle solve claim0:", o["newNodeClaims"][0].get("requirementsString"), o["newNodeClaims"][0]["pods"])
            if gs["newNodeClaims"]:
                print("   gpu    solve claim0:", gs["newNodeClaims"][0].get("requirementsString"), gs["newNodeClaims"][0]["pods"])
            print("   oracle sim:", json.dumps(w)[:400])
            print("   gpu sim   :", json.dumps(g)[:400])
            for k in ("newNodeClaims", "existingNodes", "podErrors"):
                if o.get(k) != gs.get(k):
                    print("   solve differs in", k)
                    print("     oracle:", json.dumps(o.get(k))[:1500])
                    print("     gpu   :", json.dumps(gs.get(k))[:1500])
    print("commands equal:", want["multi"]["command"] == res["tact"]["multi"]["command"],
          want["single"]["command"] == res["tact"]["single"]["command"])


if __name__ == "__main__":
    main()
