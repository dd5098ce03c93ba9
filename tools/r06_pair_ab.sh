#!/bin/bash
# r06: tile pairs sharing their D1 sign words in the two-blocks-per-CU row
# passes (apply_signs_pair) vs unpaired (OFL_EDEN_PAIR=0): -m gpu suite first,
# then the Llama step, the 1 GiB set and ResNet-50 alternated, three rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_pair; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b l_pair_$r X=1 -- --steps 8 --warmup 2
  b l_nopair_$r OFL_EDEN_PAIR=0 -- --steps 8 --warmup 2
  b u_pair_$r X=1 -- --workload uniform_1gib --steps 30 --warmup 5
  b u_nopair_$r OFL_EDEN_PAIR=0 -- --workload uniform_1gib --steps 30 --warmup 5
  b rn_pair_$r X=1 -- --workload resnet50_fp32 --steps 300 --warmup 20
  b rn_nopair_$r OFL_EDEN_PAIR=0 -- --workload resnet50_fp32 --steps 300 --warmup 20
done
