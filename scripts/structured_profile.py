#!/usr/bin/env python3
"""Where a drop-in Solve's return path spends its time on C2.

Usage: KS_HOST_TIMING=1 python scripts/structured_profile.py   (collect()'s phases go to stderr)
Per step: the kernel-only Solve (timing_only), ks_solve with the Results collected, the structured
accessor walk in Python (ctypes), and ks_results_free.
"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-sigs_amd"))

from karpenter_amd import Scheduler, synth  # noqa: E402
from karpenter_amd import scheduler as ks  # noqa: E402


def main():
    import json
    sch = Scheduler(json.dumps(synth.config2(50000, 400)))
    l = ks.lib()
    for _ in range(2):
        sch.solve(timing_only=True)
        sch.solve_structured()
    for step in range(5):
        t0 = time.perf_counter()
        sch.solve(timing_only=True)
        t1 = time.perf_counter()
        o = ks._Opts(-1, 1, 1, 0, 0)
        r = ctypes.c_void_p()
        ks._check(l.ks_solve(sch._h, ctypes.byref(o), ctypes.byref(r)))
        t2 = time.perf_counter()
        claims, nodes, errors = ks._read_structured(l, r)
        t3 = time.perf_counter()
        l.ks_results_free(r)
        t4 = time.perf_counter()
        print("step %d: kernel-only solve %.3f ms | ks_solve + collect %.3f ms | python accessor walk %.3f ms "
              "(%d claims) | free %.3f ms" % (step, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, len(claims),
                                              (t4 - t3) * 1e3), flush=True)


if __name__ == "__main__":
    main()
