#!/bin/bash
# rocprofv3 evidence for the bench workloads: kernel trace + stats, then one PMC pass per counter group.
# Usage: scripts/profile.sh <tag>   (writes gpurun_out/prof_<tag>_*)
set -o pipefail
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
B="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --cons-steps 3"
S="python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --cons-steps 3 --cons-topo-apps 0"
C="python3 $R/bench.py --only-consolidation --warmup 1 --no-cpu-baseline --cons-steps 3"
out=$R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_${tag}_trace -o run -- $B > $out/prof_${tag}_trace.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/prof_${tag}_fetch -o run -- $S > $out/prof_${tag}_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/prof_${tag}_write -o run -- $S > $out/prof_${tag}_write.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $out/prof_${tag}_sq -o run -- $S > $out/prof_${tag}_sq.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/prof_${tag}_cfetch -o run -- $C > $out/prof_${tag}_cfetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/prof_${tag}_cwrite -o run -- $C > $out/prof_${tag}_cwrite.log 2>&1 || exit $?
echo profile done
