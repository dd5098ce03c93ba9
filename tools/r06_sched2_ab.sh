#!/bin/bash
# r06: 128 MiB waves on two streams with the two-blocks-per-CU row kernels
# everywhere (OFL_EDEN_ROW2=1) vs only where a wave has < 5 tiles per CU
# (OFL_EDEN_ROW2_TPC=5: the 2 GiB waves of the 2^29 slices keep the
# persistent kernels); ResNet-50 at 128 MiB waves vs its default.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_sched2; mkdir -p $O
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b l_r2all_$r OFL_EDEN_ROW2=1 -- --wave-mib 128 --streams 2 --steps 8 --warmup 2
  b l_tpc5_$r OFL_EDEN_ROW2_TPC=5 -- --wave-mib 128 --streams 2 --steps 8 --warmup 2
  b rn_def_$r X=1 -- --workload resnet50_fp32 --steps 300 --warmup 20
  b rn_w128_$r OFL_EDEN_ROW2_TPC=5 -- --workload resnet50_fp32 --wave-mib 128 --streams 2 --steps 300 --warmup 20
done
