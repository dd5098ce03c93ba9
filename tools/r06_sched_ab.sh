#!/bin/bash
# r06: MALL-sized waves (two-blocks-per-CU rows, two streams) vs the default
# schedule, after the additive-LCG signs: the Llama step and the 1 GiB set,
# alternated, three rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_sched; mkdir -p $O
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  b l_def_$r X=1 -- --steps 8 --warmup 2
  b l_w128_$r OFL_EDEN_ROW2=1 -- --wave-mib 128 --streams 2 --steps 8 --warmup 2
  b l_w256_$r OFL_EDEN_ROW2=1 -- --wave-mib 256 --streams 2 --steps 8 --warmup 2
  b u_def_$r X=1 -- --workload uniform_1gib --steps 30 --warmup 5
  b u_w128_$r OFL_EDEN_ROW2=1 -- --workload uniform_1gib --wave-mib 128 --streams 2 --steps 30 --warmup 5
  b u_w256_$r OFL_EDEN_ROW2=1 -- --workload uniform_1gib --wave-mib 256 --streams 2 --steps 30 --warmup 5
done
