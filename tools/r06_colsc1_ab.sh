#!/bin/bash
# r06: the product with sc1 intermediate stores (default): the -m gpu suite and
# smoke first; then the column body's pointer stores sc1 as well
# (abvar/libofl_colsc1.so, -DOFL_COL_SC1=1: the 2^29 slices' outer passes,
# ResNet-50's small middle passes) vs the product, alternated x3.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_colsc1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
tail -1 $O/smoke.log
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  for v in prod colsc1; do
    if [ $v = prod ]; then e=X=1; else e=OFL_CODEC_LIB=$R/abvar/libofl_$v.so; fi
    b l_${v}_$r $e -- --steps 8 --warmup 2
    b rn_${v}_$r $e -- --workload resnet50_fp32 --steps 300 --warmup 20
  done
done
b u_prod_1 X=1 -- --workload uniform_1gib --steps 30 --warmup 5
