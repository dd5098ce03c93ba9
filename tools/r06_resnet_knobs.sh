#!/bin/bash
# r06: ResNet-50 knobs under the final cache policies: the fused small-set
# column launch (default) vs the small-set launch beside it on a side stream
# (OFL_EDEN_FUSESET=0), and tile pairs off (OFL_EDEN_PAIR=0: 780 row tiles,
# 390 pairs underfill the 512 block slots), alternated x3.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_resnet_knobs; mkdir -p $O
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b rn_def_$r X=1 -- --workload resnet50_fp32 --steps 300 --warmup 20
  b rn_nofuse_$r OFL_EDEN_FUSESET=0 -- --workload resnet50_fp32 --steps 300 --warmup 20
  b rn_nopair_$r OFL_EDEN_PAIR=0 -- --workload resnet50_fp32 --steps 300 --warmup 20
done
