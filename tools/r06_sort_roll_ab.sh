#!/bin/bash
# r06: largest-first wave packing (OFL_EDEN_WAVESORT=1: one slice size per
# wave, one column launch) and k_dec_rowA2's rolling plane prefetch
# (OFL_EDEN_DECA_ROLL=1) vs the current default: the -m gpu suite with both on
# first, then the Llama step / 1 GiB set / ResNet-50, alternated, three rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_sortroll; mkdir -p $O
OFL_EDEN_WAVESORT=1 OFL_EDEN_DECA_ROLL=1 timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu_both.log 2>&1
rc=$?; echo "pytest (both on) rc=$rc"; tail -2 $O/pytest_gpu_both.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b l_def_$r X=1 -- --steps 8 --warmup 2
  b l_sort_$r OFL_EDEN_WAVESORT=1 -- --steps 8 --warmup 2
  b l_roll_$r OFL_EDEN_DECA_ROLL=1 -- --steps 8 --warmup 2
  b l_both_$r OFL_EDEN_WAVESORT=1 OFL_EDEN_DECA_ROLL=1 -- --steps 8 --warmup 2
  b u_def_$r X=1 -- --workload uniform_1gib --steps 30 --warmup 5
  b u_roll_$r OFL_EDEN_DECA_ROLL=1 -- --workload uniform_1gib --steps 30 --warmup 5
  b rn_def_$r X=1 -- --workload resnet50_fp32 --steps 300 --warmup 20
  b rn_roll_$r OFL_EDEN_DECA_ROLL=1 -- --workload resnet50_fp32 --steps 300 --warmup 20
done
