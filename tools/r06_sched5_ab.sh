#!/bin/bash
# r06: wave size once more with sc1 intermediate stores (cheaper launch
# boundaries): 128 (default) vs 64 / 96 MiB on two streams, Llama-3-8B and the
# 1 GiB set, alternated x2; first the parity subset and ResNet-50 on the
# product with sc1 stores in col_body's middle passes.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_sched5; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "schedules or row2 or golden or small_set or fused" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2; do
  b rn_$r X=1 -- --workload resnet50_fp32 --steps 300 --warmup 20
done
for r in 1 2; do
  for w in 128 64 96; do
    b l_w${w}_$r X=1 -- --wave-mib $w --streams 2 --steps 8 --warmup 2
    b u_w${w}_$r X=1 -- --workload uniform_1gib --wave-mib $w --streams 2 --steps 30 --warmup 5
  done
done
