#!/usr/bin/env python3
"""Per-kernel resource usage of the built gfx950 code objects: SGPR / VGPR / AGPR counts,
SGPR and VGPR spill counts, scratch (private segment) bytes, LDS, and code size, read from each
translation unit's AMDGPU metadata (.hip_fatbin section -> clang-offload-bundler -> llvm-readelf --notes).
CPU only; the numbers are those of the objects the shipped libkarpenter_amd.so links.

    python scripts/resource_usage.py [out.txt]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "karpenter-sigs_amd", "build")
LLVM = "/opt/rocm/lib/llvm/bin"
TUS = ["ks_solve", "ks_solve_topo", "ks_sim", "ks_sim_topo", "ks_queue"]
FIELDS = [".sgpr_count", ".sgpr_spill_count", ".vgpr_count", ".agpr_count", ".vgpr_spill_count",
          ".private_segment_fixed_size", ".group_segment_fixed_size"]


def kernels(obj):
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb.bin"), os.path.join(td, "co.o")
        subprocess.check_call(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb])
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fb, "--output=" + co])
        notes = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", co], text=True)
        syms = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "-sW", co], text=True)
    sizes = {}
    for line in syms.splitlines():
        p = line.split()
        if len(p) >= 8 and p[3] == "FUNC":
            sizes[p[7]] = int(p[2])
    out, cur = [], None
    for line in notes.splitlines():
        s = line.strip().lstrip("- ").strip()
        if ":" not in s:
            continue
        k, v = [x.strip() for x in s.split(":", 1)]
        if k == ".agpr_count" and line.strip().startswith("-"):
            cur = {}
            out.append(cur)
        if cur is None:
            continue
        if k in FIELDS:
            cur[k] = int(v)
        elif k == ".name":
            cur["name"] = v
    for k in out:
        k["code_bytes"] = sizes.get(k.get("name", ""), 0)
    return [k for k in out if "name" in k]


def pretty(mangled):
    m = re.match(r"_ZN2ks7k_solveILi(\d)ELb(\d)ELb(\d)ELb(\d)ELb(\d)E", mangled)
    if m:
        rt, tl, sim, topo, lean = m.groups()
        return "k_solve<RT=%s,TL=%s,SIM=%s,TOPO=%s,LEAN=%s>" % (rt, tl, sim, topo, lean)
    try:
        return subprocess.check_output(["c++filt", mangled], text=True).strip()[:90]
    except OSError:
        return mangled[:90]


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else None
    head = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], text=True).strip()
    lines = ["# kernel resource usage, gfx950 objects under karpenter-sigs_amd/build (HEAD %s)" % head,
             "# sgpr/vgpr/agpr: registers allocated; *_spill: spilled registers (SGPR spills go to VGPR lanes via",
             "# v_writelane/v_readlane, VGPR spills to scratch); scratch: private segment bytes per lane; lds: static",
             "# LDS bytes (k_solve's dynamic LDS plan is per launch, make_plan)",
             "%-14s %-46s %5s %6s %5s %5s %6s %7s %6s %7s" % ("unit", "kernel", "sgpr", "sspill", "vgpr", "agpr", "vspill",
                                                              "scratch", "lds", "code_B")]
    for tu in TUS:
        obj = os.path.join(BUILD, tu + ".o")
        if not os.path.exists(obj):
            continue
        for k in kernels(obj):
            if "ks" not in k["name"]:  # (the hipCUB radix-sort kernels ks_queue.hip instantiates)
                continue
            lines.append("%-14s %-46s %5d %6d %5d %5d %6d %7d %6d %7d" % (
                tu, pretty(k["name"]), k.get(".sgpr_count", 0), k.get(".sgpr_spill_count", 0), k.get(".vgpr_count", 0),
                k.get(".agpr_count", 0), k.get(".vgpr_spill_count", 0), k.get(".private_segment_fixed_size", 0),
                k.get(".group_segment_fixed_size", 0), k["code_bytes"]))
    text = "\n".join(lines) + "\n"
    if out:
        with open(out, "w") as f:
            f.write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
