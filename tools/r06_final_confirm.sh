#!/bin/bash
# r06 last call: the final tree's -m gpu suite and smoke, the default bench
# line three times, and k_enc_rowC2's rolling prefetch off (OFL_EDEN_ROLL=0)
# vs on at the MALL-sized waves (Llama-3-8B / 1 GiB set, alternated x2).
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_final_confirm; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 11
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12
tail -1 $O/smoke.log
for r in 1 2 3; do
  timeout -k 10 600 python -u bench.py > $O/bench_$r.json 2> $O/bench_$r.err || exit 13
  echo "bench_$r $(python -c "import json;d=json.load(open('$O/bench_$r.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],{k:v.get('value') for k,v in d['also'].items() if isinstance(v,dict)})")"
done
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2; do
  b l_roll_$r X=1 -- --steps 8 --warmup 2
  b l_noroll_$r OFL_EDEN_ROLL=0 -- --steps 8 --warmup 2
  b u_roll_$r X=1 -- --workload uniform_1gib --steps 30 --warmup 5
  b u_noroll_$r OFL_EDEN_ROLL=0 -- --workload uniform_1gib --steps 30 --warmup 5
done
