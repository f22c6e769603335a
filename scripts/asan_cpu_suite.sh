#!/bin/bash
# The CPU test suite (pytest -m "not gpu") against the ASan + UBSan builds of the host translation units
# (libkarpenter_amd_asan.so) and of the oracle (liboracle_asan.so).  Python itself is not instrumented, so
# libasan / libubsan are preloaded.  Leak checking is off (the interpreter's own allocations).
set -euo pipefail
cd "$(dirname "$0")/.."
# the instrumented libraries are large and no GPU run loads them: removed again when the run ends
trap 'rm -f karpenter-sigs_amd/karpenter_amd/libkarpenter_amd_asan.so oracle/_build/liboracle_asan.so' EXIT
make -s -j8 -C karpenter-sigs_amd asan
make -s -j8 -C oracle asan
export KS_LIB_VARIANT=asan KS_ORACLE_VARIANT=asan
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
  python -m pytest tests -q -x -m "not gpu" -p no:cacheprovider "$@"
