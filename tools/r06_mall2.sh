#!/bin/bash
# r06: the product kernels at MALL-sized waves without per-launch events:
# the persistent one-block-per-CU row kernels (register prefetch of the next
# tile; OFL_EDEN_ROW2=0) against the two-blocks-per-CU ones (=1), two streams;
# and the per-tile row tables (OFL_EDEN_BTAB=0: the prefix search) on
# ResNet-50 and the 1 GiB set.  Outputs: gpurun_out/r06_mall2/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r06_mall2
mkdir -p $O
T() { timeout -k 10 "$@"; }
run() {  # tag env... -- bench args
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 200 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2> $O/$tag.err || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['ms_per_step'],d['gpu_ms_per_step_rank0'])")"
}
for rep in 1 2; do
  for w in 64 128 256; do
    for r2 in 0 1; do
      run u_w${w}_s2_r2${r2}_$rep OFL_EDEN_ROW2=$r2 -- --workload uniform_1gib --wave-mib $w --streams 2 --steps 30 --warmup 5
    done
  done
  run u_default_$rep X=1 -- --workload uniform_1gib --steps 30 --warmup 5
  run rn_btab_$rep X=1 -- --workload resnet50_fp32 --steps 300 --warmup 20
  run rn_nobtab_$rep OFL_EDEN_BTAB=0 -- --workload resnet50_fp32 --steps 300 --warmup 20
done
echo "mall2 done"
