#!/usr/bin/env python3
"""Summarise a scripts/profile_all.sh run, one block per workload.

Usage: scripts/pmc_workloads.py <tag> [workloads...]   (reads gpurun_out/prof_<tag>_*)

Per workload (c1 c2 c3 c4 c5 c5t) the dominant kernel is the k_solve instantiation of that process at its
largest grid (a consolidation pass, not its one-simulation validation launches).  Writes
  profiles/<tag>_<w>_pmc.txt      counters per launch (averaged over the profiled launches) + derived lines
  profiles/traffic_<w>.json       HBM bytes per launch for bench.py's roofline.traffic / hbm_frac
and copies the trace's kernel stats to profiles/<tag>_kernel_stats.csv (each workload's own trace to
profiles/<tag>_<w>_kernel_stats.csv).  k_feasibility (the Solve's feasibility matrix) gets <w>_feasibility files.
HBM bytes follow MI355X_MICROARCH.md (HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE count KiB; on gfx950
FETCH_SIZE reports half the bytes of a coalesced read, so it is doubled.  SQ_*_CYCLES count quad-cycles.
"""
import collections
import csv
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def rows(tag, w, grp):
    path = os.path.join(OUT, "prof_%s_%s_%s" % (tag, w, grp), "run_counter_collection.csv")
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def lib_sha():
    """sha256 of the library build profiled (bench.py flags a traffic figure from another build as stale)."""
    so = os.path.join(ROOT, "karpenter-sigs_amd", "karpenter_amd", "libkarpenter_amd.so")
    return hashlib.sha256(open(so, "rb").read()).hexdigest() if os.path.exists(so) else None


def main():
    tag = sys.argv[1]
    ws = sys.argv[2:] or ["c1", "c2", "c3", "c4", "c5", "c5t"]
    ks = os.path.join(OUT, "prof_%s_trace" % tag, "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(PROF, "%s_kernel_stats.csv" % tag))
    sha = lib_sha()
    for w in ws:
        wk = os.path.join(OUT, "prof_%s_%s_trace" % (tag, w), "run_kernel_stats.csv")
        if os.path.exists(wk):  # the workload's own trace: its averages alone (C1 and C2 share an instantiation)
            shutil.copy(wk, os.path.join(PROF, "%s_%s_kernel_stats.csv" % (tag, w)))
        summarise(tag, w, "k_solve", w, sha)
        summarise(tag, w, "k_feasibility<", w + "_feasibility", sha)


def summarise(tag, w, kernel, name, sha):
    """Counters per launch of `kernel`'s largest-grid instantiation in workload w's PMC passes."""
    allr = [r for g in ("fetch", "write", "sq", "sq2") for r in rows(tag, w, g) if kernel in r["Kernel_Name"]]
    if not allr:
        return
    grid = max(int(r["Grid_Size"]) for r in allr)
    names = collections.Counter(r["Kernel_Name"] for r in allr if int(r["Grid_Size"]) == grid)
    kname = names.most_common(1)[0][0]
    agg = collections.defaultdict(list)
    for r in allr:
        if r["Kernel_Name"] == kname and int(r["Grid_Size"]) == grid:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    v = {k: sum(x) / len(x) for k, x in agg.items()}
    short = kname.split("(")[0].replace("void ks::", "")
    lines = ["%s: PMC per launch of %s, grid %d work-items (%s)" % (name, short, grid, tag)]
    for k in sorted(v):
        lines.append("  %-22s %18.1f   (%d launches)" % (k, v[k], len(agg[k])))
    if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
        rd, wr = 2 * v["FETCH_SIZE"] * 1024, v["WRITE_SIZE"] * 1024
        lines.append("HBM bytes per launch: read %.0f (FETCH_SIZE x2 KiB) + write %.0f = %.0f" % (rd, wr, rd + wr))
        with open(os.path.join(PROF, "traffic_%s.json" % name), "w") as f:
            json.dump({"tag": tag, "kernel": short, "grid": grid, "hbm_read_bytes_per_launch": rd,
                       "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr, "lib_sha256": sha},
                      f, indent=1)
    if v.get("SQ_WAVE_CYCLES"):
        wc = v["SQ_WAVE_CYCLES"]
        lines.append("wave-cycle split: wait %.3f  issue-stall %.3f  active %.3f  (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / "
                     "SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES)" % (v.get("SQ_WAIT_ANY", 0) / wc,
                                                                  v.get("SQ_WAIT_INST_ANY", 0) / wc,
                                                                  v.get("SQ_ACTIVE_INST_ANY", 0) / wc))
        if v.get("SQ_WAVES"):
            lines.append("per wave: %.0f quad-cycles (%.0f cycles)" % (wc / v["SQ_WAVES"], 4 * wc / v["SQ_WAVES"]))
    if v.get("SQ_INSTS_VALU") is not None and v.get("SQ_WAVES"):
        n = v["SQ_WAVES"]
        lines.append("instructions per wave: VALU %.0f  SALU %.0f  SMEM %.0f  LDS %.0f  VMEM %.0f" % (
            v["SQ_INSTS_VALU"] / n, v.get("SQ_INSTS_SALU", 0) / n, v.get("SQ_INSTS_SMEM", 0) / n,
            v.get("SQ_INSTS_LDS", 0) / n, v.get("SQ_INSTS_VMEM", 0) / n))
        if v.get("SQ_WAVE_CYCLES"):
            wc = v["SQ_WAVE_CYCLES"]
            lines.append("active share: VALU %.3f  SALU %.3f  LDS %.3f (SQ_ACTIVE_INST_* over SQ_WAVE_CYCLES)" % (
                v.get("SQ_ACTIVE_INST_VALU", 0) / wc, v.get("SQ_ACTIVE_INST_SALU", 0) / wc,
                v.get("SQ_ACTIVE_INST_LDS", 0) / wc))
    txt = "\n".join(lines) + "\n"
    with open(os.path.join(PROF, "%s_%s_pmc.txt" % (tag, name)), "w") as f:
        f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
