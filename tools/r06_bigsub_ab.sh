#!/bin/bash
# r06: sub-wave size of the split 2^29 slices: the wave size (128 MiB,
# default) vs 64 and 256 MiB (OFL_EDEN_BIGSUB_MIB), Llama-3-8B alternated x3.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_bigsub; mkdir -p $O
OFL_EDEN_BIGSUB_MIB=64 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "five_pass or 2p29" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b l_sub128_$r X=1 -- --steps 8 --warmup 2
  b l_sub64_$r OFL_EDEN_BIGSUB_MIB=64 -- --steps 8 --warmup 2
  b l_sub256_$r OFL_EDEN_BIGSUB_MIB=256 -- --steps 8 --warmup 2
done
