#!/bin/bash
# ThreadSanitizer over the threaded host code (ks_parallel.h workers, the JSON parser's parallel arrays,
# NewTopology's per-pod groups, consolidation's pod parse, the snapshot reaper thread): the TSan build of the
# host objects (make tsan) driven by a fully instrumented C++ harness (scripts/tsan_host_main.cpp) over
# snapshots large enough that every parallel_for splits across 8 threads.  Any report aborts the run.
set -euo pipefail
cd "$(dirname "$0")/.."
trap 'rm -rf karpenter-sigs_amd/karpenter_amd/libkarpenter_amd_tsan.so /tmp/ks_tsan' EXIT
make -s -j8 -C karpenter-sigs_amd tsan
mkdir -p /tmp/ks_tsan
LIB=$PWD/karpenter-sigs_amd/karpenter_amd
g++ -O1 -g -fsanitize=thread scripts/tsan_host_main.cpp -o /tmp/ks_tsan/run -L"$LIB" -lkarpenter_amd_tsan \
  -Wl,-rpath,"$LIB" -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
python3 - <<'PY'
import json, sys
sys.path[:0] = [".", "karpenter-sigs_amd"]
from karpenter_amd import synth
snaps = {"c2_20k": synth.config2(20000), "c4_3000x600": synth.config4(3000, 600),
         "c3_3000": synth.config3(3000), "c5_1000": synth.config5(1000),
         "c5t_400": synth.cluster_snapshot(400, 20, 400, seed=4205, topology=8)}
for k, v in snaps.items():
    open("/tmp/ks_tsan/%s.json" % k, "w").write(json.dumps(v))
PY
export KS_HOST_THREADS=8 TSAN_OPTIONS="halt_on_error=1:exitcode=66:second_deadlock_stack=1"
for s in c2_20k c4_3000x600 c3_3000; do /tmp/ks_tsan/run solve /tmp/ks_tsan/$s.json; done
for s in c5_1000 c5t_400; do /tmp/ks_tsan/run cons /tmp/ks_tsan/$s.json; done
echo "tsan host: no reports"
