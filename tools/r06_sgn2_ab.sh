#!/bin/bash
# r06: D1 sign bitmaps written by blocks appended to an earlier row launch of
# the same stream (no launch of their own) vs per-element hashes
# (OFL_EDEN_SGN=0); the Eden parity tests first.  1 GiB set and Llama at
# 128 MiB waves on two streams (two-blocks-per-CU row kernels), ResNet-50
# default, the default 2 GiB-wave Llama step; alternated, two rounds.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r06_sgn2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -n 2 $O/parity.log; [ $rc -eq 0 ] || exit 1
b() {  # tag env -- args
  local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2> $O/$tag.err || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'],d['check_rel_l2'])")"
}
for rep in 1 2; do
  for sg in 1 0; do
    b rn_s${sg}_$rep OFL_EDEN_SGN=$sg -- --workload resnet50_fp32 --steps 300 --warmup 20
    b u128_s${sg}_$rep OFL_EDEN_SGN=$sg OFL_EDEN_ROW2=1 -- --workload uniform_1gib --wave-mib 128 --streams 2 --steps 30 --warmup 5
    b u64_s${sg}_$rep OFL_EDEN_SGN=$sg OFL_EDEN_ROW2=1 -- --workload uniform_1gib --wave-mib 64 --streams 2 --steps 30 --warmup 5
    b l128_s${sg}_$rep OFL_EDEN_SGN=$sg OFL_EDEN_ROW2=1 -- --wave-mib 128 --streams 2 --steps 8 --warmup 2
  done
  b ldef_$rep X=1 -- --steps 8 --warmup 2
done
