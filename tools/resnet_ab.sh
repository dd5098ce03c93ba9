#!/bin/bash
# ResNet-50 step A/B of library variants (OFL_CODEC_LIB), alternating runs:
#   bash tools/resnet_ab.sh OUT_DIR RUNS lib_a.so [lib_b.so ...]   ("default" = in-tree build)
set -euo pipefail
O=$1; N=$2; shift 2
mkdir -p "$O"
WL=${AB_WORKLOAD:-resnet50_fp32}
for i in $(seq "$N"); do
  for L in "$@"; do
    tag=$(basename "$L" .so)
    if [ "$L" = default ]; then unset OFL_CODEC_LIB; else export OFL_CODEC_LIB=$L; fi
    timeout -k 10 180 python bench.py --workload "$WL" --no-cpu-baseline --also= --steps ${AB_STEPS:-200} --warmup 10 \
        ${AB_ARGS:-} > "$O/${tag}_$i.json" 2> "$O/${tag}_$i.err"
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$O/${tag}_$i.json" "$tag"
  done
done
