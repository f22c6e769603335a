#!/bin/bash
# rocprofv3 evidence for every bench workload on the build being benched:
#   trace : kernel trace + stats of the default bench command (minus the CPU baseline legs), so the kernel
#           averages are those of the timed launches;
#   then per workload (C1, C2, C3, C4, C5, C5T, one bench process each): PMC passes FETCH_SIZE, WRITE_SIZE
#   (HBM bytes, corrected per MI355X_MICROARCH.md in scripts/pmc_summary.py), and two SQ passes (wave cycles,
#   wait / issue / active split; instruction mix).  Counters never share a pass with a trace domain.
# Usage: scripts/profile_all.sh <tag> [workloads...]   (writes gpurun_out/prof_<tag>_*)
set -o pipefail
tag=${1:-r04}
shift
W=${@:-c1 c2 c3 c4 c5 c5t}
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
out=$R/gpurun_out
P="python3 $R/bench.py --warmup 1 --no-cpu-baseline --no-shards --cons-steps 3 --steps 3"
cmd_for() {
  case $1 in
    c1|c2|c3|c4) echo "$P --only-solve $1" ;;
    c5) echo "$P --only-consolidation --cons-topo-apps 0" ;;
    c5t) echo "$P --only-consolidation --no-c5" ;;
  esac
}
if [ -z "$NO_TRACE" ]; then  # NO_TRACE=1: only the per-workload passes (a second call for the remaining workloads)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_${tag}_trace -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/prof_${tag}_trace.log 2>&1 || exit $?
fi
for w in $W; do
  C=$(cmd_for $w)
  # the workload's own kernel trace: per-workload averages (C1 and C2 launch the same instantiation)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_${tag}_${w}_trace -o run -- $C > $out/prof_${tag}_${w}_trace.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/prof_${tag}_${w}_fetch -o run -- $C > $out/prof_${tag}_${w}_fetch.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/prof_${tag}_${w}_write -o run -- $C > $out/prof_${tag}_${w}_write.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $out/prof_${tag}_${w}_sq -o run -- $C > $out/prof_${tag}_${w}_sq.log 2>&1 || exit $?
done
for w in $W; do
  C=$(cmd_for $w)
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS --output-format csv -d $out/prof_${tag}_${w}_sq2 -o run -- $C > $out/prof_${tag}_${w}_sq2.log 2>&1 || exit $?
done
echo profile done
