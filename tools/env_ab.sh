#!/bin/bash
# Step A/B of one env setting over values, alternating runs, on a workload:
#   bash tools/env_ab.sh OUT_DIR RUNS WORKLOAD VAR v1 v2 ...   ("-" = unset)
set -euo pipefail
O=$1; N=$2; WL=$3; VAR=$4; shift 4
mkdir -p "$O"
for i in $(seq "$N"); do
  for v in "$@"; do
    if [ "$v" = - ]; then unset "$VAR"; else export "$VAR=$v"; fi
    timeout -k 10 180 python bench.py --workload "$WL" --no-cpu-baseline --also= --steps ${AB_STEPS:-200} --warmup 10 \
        --no-kernel-events ${AB_ARGS:-} > "$O/${WL}_${v}_$i.json" 2> "$O/${WL}_${v}_$i.err"
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['gpu_ms_per_step_rank0'])" "$O/${WL}_${v}_$i.json" "$WL $VAR=$v"
  done
done
unset "$VAR"
