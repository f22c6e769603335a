#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run: per-launch kernel stats + PMC counters for one kernel.

Usage: scripts/pmc_summary.py <tag> [kernel_substring] [traffic_name] [min_grid] [max_grid]   (reads gpurun_out/prof_<tag>_*)
Writes profiles/<tag>_kernel_stats.csv, profiles/<tag>_<traffic_name>_pmc.txt and profiles/traffic_<traffic_name>.json.
min_grid: only launches with at least that many work-items (a consolidation pass, not its one-simulation
validation launches of the same kernel).
HBM bytes follow MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB; on gfx950
FETCH_SIZE reports half the bytes of a coalesced read, so it is doubled.
"""
import collections
import csv
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    kname = sys.argv[2] if len(sys.argv) > 2 else "k_solve"
    tname = sys.argv[3] if len(sys.argv) > 3 else "c2"
    min_grid = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    max_grid = int(sys.argv[5]) if len(sys.argv) > 5 else 1 << 62
    out = os.path.join(ROOT, "gpurun_out")
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(out, "prof_%s_trace" % tag, "run_kernel_stats.csv"),
                os.path.join(prof, "%s_kernel_stats.csv" % tag))
    lines = ["PMC per launch of %s (averaged over the profiled launches%s)" % (
        kname, ", grid >= %d" % min_grid if min_grid else "")]
    vals = {}
    agg = collections.defaultdict(list)
    for grp in ("fetch", "write", "sq", "cfetch", "cwrite"):
        path = os.path.join(out, "prof_%s_%s" % (tag, grp), "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for r in csv.DictReader(open(path)):
            if kname in r["Kernel_Name"] and min_grid <= int(r["Grid_Size"]) <= max_grid:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        vals[k] = sum(v) / len(v)
        lines.append("  %-22s %16.1f   (%d launches)" % (k, vals[k], len(v)))
    if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
        rd = 2 * vals["FETCH_SIZE"] * 1024
        wr = vals["WRITE_SIZE"] * 1024
        lines.append("HBM bytes per launch: read %.0f (FETCH_SIZE x2 KiB) + write %.0f = %.0f" % (rd, wr, rd + wr))
        # the build profiled (bench.py flags the figure stale when the library it loads differs)
        so = os.path.join(ROOT, "karpenter-sigs_amd", "karpenter_amd", "libkarpenter_amd.so")
        lib_sha = hashlib.sha256(open(so, "rb").read()).hexdigest() if os.path.exists(so) else None
        with open(os.path.join(prof, "traffic_%s.json" % tname), "w") as f:
            json.dump({"tag": tag, "kernel": kname, "hbm_read_bytes_per_launch": rd,
                       "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
                       "lib_sha256": lib_sha}, f, indent=1)
    if "SQ_WAVE_CYCLES" in vals and "SQ_BUSY_CYCLES" in vals:
        lines.append("SQ_WAIT_ANY / SQ_WAVE_CYCLES = %.3f ; SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES = %.3f" % (
            vals.get("SQ_WAIT_ANY", 0) / vals["SQ_WAVE_CYCLES"], vals.get("SQ_ACTIVE_INST_ANY", 0) / vals["SQ_WAVE_CYCLES"]))
    txt = "\n".join(lines) + "\n"
    with open(os.path.join(prof, "%s_%s_pmc.txt" % (tag, tname)), "w") as f:
        f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
