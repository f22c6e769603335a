#!/bin/bash
# Run one GPU test selection against each library variant (KS_LIB_VARIANT), one pytest process each.
# Usage: scripts/variant_check.sh "<pytest args>" variant...   ("" = the main build)
sel="$1"; shift
for v in "$@"; do
  echo "=== variant '${v}'"
  KS_LIB_VARIANT="$v" timeout -k 10 300 python -u -m pytest $sel -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -n 4
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
