#!/bin/bash
# The C5T consolidation line (pass ms, kernel ms, update + pass) for each library variant (KS_LIB_VARIANT),
# one bench process each.  Usage: scripts/variant_bench.sh variant...   ("" = the main build)
mkdir -p gpurun_out
for v in "$@"; do
  echo "=== variant '${v}'"
  KS_LIB_VARIANT="$v" timeout -k 10 300 python -u bench.py --only-consolidation --no-cpu-baseline --no-c5 --no-shards \
    > "gpurun_out/vb_${v:-main}.json" 2> "gpurun_out/vb_${v:-main}.err"
  rc=$?
  python - "gpurun_out/vb_${v:-main}.json" <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    for x in [d] + [v for v in d.values() if isinstance(v, dict) and "ms_per_pass" in v]:
        if "ms_per_pass" in x:
            u = x.get("incremental_update", {})
            print(x["metric"][:60], "pass", x["ms_per_pass"], "kernel", x["roofline"].get("kernel_ms"),
                  "upd+pass", u.get("update_plus_pass_ms"), "upd", u.get("update_ms"), "pau", u.get("pass_after_update_ms"))
EOF
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; tail -5 "gpurun_out/vb_${v:-main}.err"; exit $rc; fi
done
