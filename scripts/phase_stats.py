#!/usr/bin/env python3
"""Diagnostic: per-phase cycle shares of k_solve (KS_LIB_VARIANT=stats build, s_memtime stamps).
Never used for timing numbers; read the SHARES, not the totals."""
import json
import os
import sys

os.environ["KS_LIB_VARIANT"] = "stats"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "karpenter-sigs_amd"))
from karpenter_amd import Scheduler, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50000
cfg = sys.argv[2] if len(sys.argv) > 2 else "c2"
snap = {"c2": lambda: synth.config2(n), "c3": lambda: synth.config3(n), "c4": lambda: synth.config4(n, max(n // 5, 1))}[cfg]()
r = Scheduler(json.dumps(snap)).solve()
st = r.stats
tot = max(st["cycTotal"], 1)
print(json.dumps(st))
for k in ["cycPop", "cycNodes", "cycNodeCommit", "cycSort", "cycQuick", "cycFull", "cycFullRs", "cycFullThr",
          "cycFullMasks", "cycFullApply", "cycCommit", "cycTemplates"]:
    print("%-14s %6.1f%%  %8.1f cyc/pod" % (k, 100.0 * st[k] / tot, st[k] / n))
print("total cyc/pod %.1f  pops %d  sorts %d slow %d  claims %d  solve_kernel_ms %.2f" % (
    tot / n, st["pops"], st["sorts"], st["sortsWithDescent"], st["nclaims"], r.solve_kernel_ms))
