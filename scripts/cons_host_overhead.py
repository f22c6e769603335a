#!/usr/bin/env python3
"""Diagnostic: where a C5 consolidation pass's wall time goes beside the kernel (bench.py's ms_per_pass vs
kernel_ms): Consolidator.run (sort + simulations + record download), needed_sims, decide."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-sigs_amd"))
from karpenter_amd import Consolidator, synth  # noqa: E402

c = Consolidator(json.dumps(synth.config5(5000)))
for _ in range(3):
    recs, _ = c.run(0, 1)
    c.decide(recs, 1, candidates=False)
rows = []
for _ in range(20):
    t0 = time.perf_counter()
    recs, k = c.run(0, 1)
    t1 = time.perf_counter()
    need = c.needed_sims(recs, 1)
    t2 = time.perf_counter()
    doc = c.decide(recs, 1, candidates=False)
    t3 = time.perf_counter()
    rows.append(((t1 - t0) * 1e3, k, (t2 - t1) * 1e3, (t3 - t2) * 1e3, len(need), len(json.dumps(doc))))
med = lambda i: sorted(r[i] for r in rows)[len(rows) // 2]  # noqa: E731
print("run wall %.3f ms (kernel events %.3f ms) | needed_sims %.3f ms (%d sims) | decide %.3f ms (doc %d B)" % (
    med(0), med(1), med(2), rows[-1][4], med(3), rows[-1][5]))
# the bench's pass (world 1): records kept in the handle's pinned buffer, decide without the per-simulation lists
rows = []
for _ in range(30):
    t0 = time.perf_counter()
    _, k = c.run(0, 1, keep=True)
    t1 = time.perf_counter()
    doc = c.decide(None, 1, candidates=False, sims=False)
    t2 = time.perf_counter()
    rows.append(((t1 - t0) * 1e3, k, (t2 - t1) * 1e3, len(json.dumps(doc))))
print("bench pass: run(keep) wall %.3f ms (kernel events %.3f ms) | decide(sims=False) %.3f ms (doc %d B)" % (
    med(0), med(1), med(2), rows[-1][3]))
