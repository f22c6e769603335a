#!/bin/bash
# Run every reproducer variant built next to this script (repro_*), each under its own time limit.
cd "$(dirname "$0")"
for b in repro_*; do
  [ -x "$b" ] || continue
  timeout -k 5 30 "./$b" || { echo "$b rc=$?"; exit 1; }
done
