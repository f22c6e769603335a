"""Per-simulation solve counters of a small consolidation cluster (debugging aid, not a test).
Usage: python scripts/cons_sim_counters.py <seed> <candidate names...>"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "karpenter-sigs_amd"))
import carry_scenarios as cs  # noqa: E402
from oracle import bridge  # noqa: E402

NAMES = ["nclaims", "nlog", "hostctr", "error", "pops", "algbytes", "sorts", "sort_slow", "claim_full",
         "claim_quick_fail", "windows"]


def main():
    seed = int(sys.argv[1])
    snap = cs.random_cluster(seed, topology=True)
    if len(sys.argv) > 2:
        snap["candidates"] = sys.argv[2:]
    from karpenter_amd import Consolidator
    s = json.dumps(snap)
    want, _ = bridge.consolidate(s, all_sims=True)
    c = Consolidator(s)
    recs, _ = c.run(0, 1)
    got = c.decide(bytes(recs), 1, all_sims=True)
    for i in range(c.num_sims):
        ctr = c.sim_counters(i)
        print("sim", i, dict(zip(NAMES, ctr[:11])))
    print("oracle single:", json.dumps(want["single"]["sims"])[:1500])
    print("gpu    single:", json.dumps(got["single"]["sims"])[:1500])


if __name__ == "__main__":
    main()
