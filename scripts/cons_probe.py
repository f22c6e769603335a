#!/usr/bin/env python3
"""Probe: C5 consolidation on one GPU (create time, run time per pass, outcome summary)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-sigs_amd"))
from karpenter_amd import Consolidator, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
t = time.time()
topo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
snap = json.dumps(synth.config5(n) if not topo else synth.cluster_snapshot(n, 20, 400, seed=4205, topology=topo))
t1 = time.time()
c = Consolidator(snap)
t2 = time.time()
print("snapshot %.2fs (%d MB) create %.2fs sims %d" % (t1 - t, len(snap) >> 20, t2 - t1, c.num_sims), flush=True)
for i in range(4):
    t = time.time()
    recs, ms = c.run()
    print("run %d: kernel %.3f ms wall %.3f ms" % (i, ms, (time.time() - t) * 1e3), flush=True)
doc = c.decide(recs, 1, all_sims=True)
acts = {}
for s in doc["single"]["sims"]:
    k = (s["allNonPendingScheduled"], s["newNodeClaims"])
    acts[k] = acts.get(k, 0) + 1
print("single outcomes", acts)
print("multi", doc["multi"]["command"]["action"], len(doc["multi"]["command"]["candidates"]))
print("single", doc["single"]["command"]["action"], doc["single"]["command"]["candidates"])
if os.environ.get("KS_LIB_VARIANT") == "stats":
    names = ["nclaims", "ncommits", "hostCtr", "error", "pops", "algBytes", "sorts", "sortSlow", "claimFull",
             "quickFail", "windows", "cycPop", "cycNodes", "cycSort", "cycQuick", "cycFull", "cycCommit", "cycTpl",
             "cycTotal", "cycNodeCommit"]
    for sim in (0, 50, 99, 100, 2000):
        if sim >= c.num_sims:
            continue
        ct = c.sim_counters(sim)
        d = dict(zip(names, ct))
        pops = max(d["pops"], 1)
        print("sim %d: pops %d total %.0f cyc/pod | pop %.0f nodes %.0f (commit %.0f) claims %.0f tpl %.0f" % (
            sim, d["pops"], d["cycTotal"] / pops, d["cycPop"] / pops, d["cycNodes"] / pops, d["cycNodeCommit"] / pops,
            (d["cycQuick"] + d["cycFull"] + d["cycCommit"] + d["cycSort"]) / pops, d["cycTpl"] / pops))
