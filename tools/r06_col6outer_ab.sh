#!/bin/bash
# r06: k_col6 for the 5-pass slices' level-1 column passes (OFL_EDEN_COL6_OUTER=7:
# the Llama 2^29 slices' k_col<7, false> sub-wave launches) vs k_col: the
# five-pass / schedule / row tests with it first, then the Llama step x3;
# also OFL_EDEN_BIGLAST=1 (the second 2^29 wave at the end of its stream;
# removed after this A/B, profiles/r06_col6outer_biglast_ab.txt).
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_col6outer; mkdir -p $O
OFL_EDEN_COL6_OUTER=7 OFL_EDEN_BIGLAST=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "five_pass or 2p29 or schedules or row2 or golden or oracle" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b l_col_$r X=1 -- --steps 8 --warmup 2
  b l_col6_$r OFL_EDEN_COL6_OUTER=7 -- --steps 8 --warmup 2
  b l_biglast_$r OFL_EDEN_BIGLAST=1 -- --steps 8 --warmup 2
done
