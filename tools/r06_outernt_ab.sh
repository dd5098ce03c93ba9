#!/bin/bash
# r06: the split 5-pass slices' outer column passes streaming their HBM side nt
# (k_col<7, false, NTL, NTS>: nt stores before the middle pass, nt loads after;
# default) vs the default policy
# (OFL_EDEN_OUTERNT=0): five-pass / schedule tests first, then the Llama step x3.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_outernt; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "five_pass or 2p29 or schedules or row2 or wavg" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b l_outernt_$r X=1 -- --steps 8 --warmup 2
  b l_outerdef_$r OFL_EDEN_OUTERNT=0 -- --steps 8 --warmup 2
done
