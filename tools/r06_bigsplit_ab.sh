#!/bin/bash
# r06: 5-pass slices bigger than a wave (the Llama embedding / lm_head, 2^29)
# split into MALL sub-waves for passes 1-2 and 4-5 vs whole-slice passes
# (OFL_EDEN_BIGSPLIT=0): the -m gpu suite first (five-pass slices vs the
# oracle, schedules bit-identical), then the Llama step alternated x3, and a
# kernel trace of each.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_bigsplit; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b l_split_$r X=1 -- --steps 8 --warmup 2
  b l_whole_$r OFL_EDEN_BIGSPLIT=0 -- --steps 8 --warmup 2
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --also "" --no-kernel-events > $O/prof_split.json 2> $O/prof_split.err || exit 21
echo "prof done"
