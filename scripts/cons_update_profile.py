#!/usr/bin/env python3
"""Where an incremental update + pass spends its time on C5 (ks_cons_update, then run + decide).

Usage: KS_HOST_TIMING=1 python scripts/cons_update_profile.py [nodes] [topology apps]   (phase lines go to stderr)
Prints per update: update ms, run ms (plan + kernel + record copy), kernel ms, decide ms.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "karpenter-sigs_amd"))

from karpenter_amd import Consolidator, synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    apps = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    snap = synth.config5(n) if not apps else synth.cluster_snapshot(n, 20, 400, seed=4205, topology=apps)
    c = Consolidator(json.dumps(snap))
    for _ in range(3):
        recs, _ = c.run(0, 1)
        c.decide(recs, 1, candidates=False)
    nodes = snap["stateNodes"]
    for i in range(8):
        a, b = nodes[200 + 2 * i], nodes[201 + 2 * i]
        delta = {"deletePods": [p["metadata"]["uid"] for p in a.get("pods", [])[:10]], "removeNodes": [b["name"]]}
        print("--- update %d" % i, file=sys.stderr, flush=True)
        t0 = time.perf_counter()
        c.update(delta)
        t1 = time.perf_counter()
        recs, kms = c.run(0, 1)
        t2 = time.perf_counter()
        c.decide(recs, 1, candidates=False)
        t3 = time.perf_counter()
        recs, kms2 = c.run(0, 1)
        t4 = time.perf_counter()
        print("update %d: update %.3f ms  run %.3f ms (kernel %.3f)  decide %.3f ms  | steady run %.3f ms (kernel %.3f)"
              % (i, (t1 - t0) * 1e3, (t2 - t1) * 1e3, kms, (t3 - t2) * 1e3, (t4 - t3) * 1e3, kms2), flush=True)


if __name__ == "__main__":
    main()
