#!/bin/bash
# The CPU test suite (pytest -m "not gpu") against the ThreadSanitizer build of the host translation units
# (libkarpenter_amd_tsan.so): the parallel JSON parse, pod encode and NewTopology workers (ks_parallel.h)
# and the snapshot reaper thread (ks_json.h).  Python is not instrumented, so libtsan is preloaded; the
# oracle (single-threaded checker) runs uninstrumented.
set -euo pipefail
cd "$(dirname "$0")/.."
trap 'rm -f karpenter-sigs_amd/karpenter_amd/libkarpenter_amd_tsan.so' EXIT
make -s -j8 -C karpenter-sigs_amd tsan
export KS_LIB_VARIANT=tsan KS_HOST_THREADS=${KS_HOST_THREADS:-8}
export TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1:report_signal_unsafe=0
# (test_abi_c.py compiles and runs a separate plain-C client binary and test_dist_gloo.py spawns torch gloo
# processes, neither of them the threaded host code; under a preloaded TSan runtime gcc and the spawned
# interpreters hang, so both are left to the ordinary and ASan suites)
LD_PRELOAD="$(gcc -print-file-name=libtsan.so)" \
  python -m pytest tests -q -x -m "not gpu" -p no:cacheprovider --ignore=tests/test_abi_c.py --ignore=tests/test_dist_gloo.py "$@"
