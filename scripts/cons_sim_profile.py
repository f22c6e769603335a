#!/usr/bin/env python3
"""Diagnostic: the critical path of a consolidation pass.  Runs the C5 (or C5 + topology) pass with the
KS_LIB_VARIANT=stats build and reads every simulation's counters (s_memtime stamps): the longest
simulation against the pass time, the distribution, and which simulations are the long ones.
Never used for timing numbers (the stats build is slower); read the SHARES and the ratios."""
import json
import os
import sys

os.environ.setdefault("KS_LIB_VARIANT", "stats")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-sigs_amd"))
from karpenter_amd import Consolidator, synth  # noqa: E402

NAMES = ["nclaims", "ncommits", "hostCtr", "error", "pops", "algBytes", "sorts", "sortSlow", "claimFull",
         "quickFail", "windows", "cycPop", "cycNodes", "cycSort", "cycQuick", "cycFull", "cycCommit", "cycTpl",
         "cycTotal", "cycNodeCommit", "cycFullRs", "cycFullThr", "cycFullMasks", "cycFullApply", "runs", "runPods",
         "sortsExact", "fTopoPop", "fState", "fRefill", "fWinTests", "fWinBlocks", "fRecord", "fNodeCommit", "fWinTopo"]

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
topo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
snap = json.dumps(synth.config5(n) if not topo else synth.cluster_snapshot(n, 20, 400, seed=4205, topology=topo))
c = Consolidator(snap)
ms = []
for _ in range(3):
    _, k = c.run()
    ms.append(k)
rows = []
for s in range(c.num_sims):
    d = dict(zip(NAMES, c.sim_counters(s)))
    rows.append((d["cycTotal"], s, d))
rows.sort(reverse=True)
tot = [r[0] for r in rows]
mx = tot[0]
print("pass kernel ms (stats build): %s" % ", ".join("%.3f" % x for x in ms))
print("simulations %d; cycTotal max %d, p50 %d, p90 %d, p99 %d, mean %.0f" % (
    len(tot), mx, tot[len(tot) // 2], tot[len(tot) // 10], tot[len(tot) // 100], sum(tot) / len(tot)))
print("sum of all simulations' cycles / max = %.1f (the pass cannot be shorter than its longest simulation)"
      % (sum(tot) / mx))
# the node phase split (scyc slots, shared with claim_full's sub-phases, which these simulations barely run):
# [0] the node phase up to the scan past the register window, [2] scan steps past the window, [3] their cycles
for cyc, s, d in rows[:4]:
    pops = max(d["pops"], 1)
    print("sim %5d node phase per pop: window part %.0f cyc, past-window steps %.2f, past-window cyc %.0f, commit %.0f" % (
        s, d["cycFullRs"] / pops, d["cycFullMasks"] / pops, d["cycFullApply"] / pops, d["cycNodeCommit"] / pops))
for cyc, s, d in rows[:4]:
    pops = max(d["pops"], 1)
    if "fTopoPop" in d:
        print("sim %5d fine per pop: topo_pop %.0f, state %.0f, refill %.0f, window tests %.0f (blocks %.2f, topology %.0f),"
              " record %.0f, node commit %.0f" % (s, d["fTopoPop"] / pops, d["fState"] / pops, d["fRefill"] / pops,
                                                  d["fWinTests"] / pops, d["fWinBlocks"] / pops, d["fWinTopo"] / pops,
                                                  d["fRecord"] / pops, d["fNodeCommit"] / pops))
for cyc, s, d in rows[:12]:
    pops = max(d["pops"], 1)
    print("sim %5d: cyc %9d (%.2f of max) pops %5d runs %4d (%5d pods, %.0f cyc) windows %3d (%.0f cyc) | pop %.0f nodes %.0f (commit %.0f) claims %.0f tpl %.0f per pod" % (
        s, cyc, cyc / mx, d["pops"], d.get("runs", 0), d.get("runPods", 0), d["cycFullThr"], d["windows"], d["cycFullRs"],
        d["cycPop"] / pops,
        d["cycNodes"] / pops, d["cycNodeCommit"] / pops,
        (d["cycQuick"] + d["cycFull"] + d["cycCommit"] + d["cycSort"]) / pops, d["cycTpl"] / pops))
# the multi-node prefix simulations are the first 100 (largest first)
multi = [r for r in rows if r[1] < 100]
single = [r for r in rows if r[1] >= 100]
print("multi-node prefixes: max %d mean %.0f; single-node: max %d mean %.0f" % (
    max(r[0] for r in multi), sum(r[0] for r in multi) / max(len(multi), 1), max(r[0] for r in single),
    sum(r[0] for r in single) / max(len(single), 1)))
