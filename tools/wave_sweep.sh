#!/bin/bash
# Large-slice wave size x streams sweep on one workload (GPU box):
#   bash tools/wave_sweep.sh WORKLOAD "MIB..." "STREAMS..."
# Prints one line per setting: GiB/s and ms/step (device-resident step).
set -euo pipefail
WL=${1:-uniform_1gib}; MIBS=${2:-"32 64 128 256 2048"}; STS=${3:-"1 2"}
mkdir -p gpurun_out
for s in $STS; do
  for m in $MIBS; do
    timeout -k 10 120 python bench.py --workload "$WL" --also "" --no-cpu-baseline --no-kernel-events \
        --steps 20 --warmup 3 --wave-mib "$m" --streams "$s" > gpurun_out/sweep_${WL}_${m}_${s}.json 2>&1
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); \
print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d['config']['waves'])" \
        gpurun_out/sweep_${WL}_${m}_${s}.json "$m" "$s"
  done
done
