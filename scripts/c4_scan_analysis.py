"""Why does a C4 pod's first-fit scan pass ~780 existing nodes?  Replays the oracle's C4 placement (queue order,
each pod's node) and classifies every node before the chosen one as failing on resources (Fits) or on
something else (topology: resources fit), per pod and per 64-node block.  Profiling aid, not a test."""
import json
import os
import sys
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "karpenter-sigs_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))

from cons_delta import parse_q, pod_requests  # noqa: E402
from karpenter_amd import synth  # noqa: E402
from oracle import bridge  # noqa: E402


def main():
    n_pods = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    snap = synth.config4(n_pods)
    res, _ = bridge.solve(json.dumps(snap))
    nodes = sorted(snap["stateNodes"], key=lambda n: n["name"])
    idx = {n["name"]: i for i, n in enumerate(nodes)}
    where = {}
    for e in res["existingNodes"]:
        for p in e["pods"]:
            where[p] = idx[e["name"]]
    pods = snap["pods"]
    req = [pod_requests(p) for p in pods]
    names = ["cpu", "memory", "pods"]
    order = sorted(range(len(pods)), key=lambda i: (-req[i].get("cpu", 0), -req[i].get("memory", 0), i))
    avail = np.array([[float(parse_q(n["available"].get(r, "0"))) for r in names] for n in nodes])
    used = np.zeros_like(avail)
    tot_r = tot_t = 0
    blk_r = blk_t = blk_mixed = 0
    placed = 0
    for i in order:
        if i not in where:
            continue
        j = where[i]
        q = np.array([float(req[i].get(r, 0)) for r in names])
        fits = np.all(used[:j] + q <= avail[:j], axis=1)
        tot_r += int((~fits).sum())
        tot_t += int(fits.sum())
        for b in range(0, j // 64):
            f = fits[b * 64:(b + 1) * 64]
            if not f.any():
                blk_r += 1
            elif f.all():
                blk_t += 1
            else:
                blk_mixed += 1
        used[j] += q
        placed += 1
    print(json.dumps({"pods": placed, "nodes_before_fit_per_pod": (tot_r + tot_t) / placed,
                      "fail_resources_per_pod": tot_r / placed, "fail_other_per_pod": tot_t / placed,
                      "blocks_all_resource_fail_per_pod": blk_r / placed,
                      "blocks_all_resource_fit_per_pod": blk_t / placed, "blocks_mixed_per_pod": blk_mixed / placed}))


if __name__ == "__main__":
    main()
