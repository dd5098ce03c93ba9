#!/bin/bash
# r06: the intermediates' buffer loads (row and k_col6 passes) with sc1
# (abvar/libofl_ldsc1.so, -DOFL_LD_AUX=16: L2-served, no L1 allocation) or nt
# (abvar/libofl_ldnt.so, -DOFL_LD_AUX=2) vs the default policy; parity subset
# with sc1 first; Llama-3-8B and the 1 GiB set alternated x2.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_wsld; mkdir -p $O
OFL_CODEC_LIB=$R/abvar/libofl_ldsc1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "five_pass or schedules or row2 or golden" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2; do
  for v in prod ldsc1 ldnt; do
    if [ $v = prod ]; then e=X=1; else e=OFL_CODEC_LIB=$R/abvar/libofl_$v.so; fi
    b l_${v}_$r $e -- --steps 8 --warmup 2
    b u_${v}_$r $e -- --workload uniform_1gib --steps 30 --warmup 5
  done
done
