#!/bin/bash
# r06: the schedule again after tile pairs + largest-first packing: wave size
# (64 / 128 / 192 / 256 MiB on two streams) and the order of the size classes
# (largest first = default, OFL_EDEN_WAVESORT=2 smallest first: the two 2^29
# waves last), Llama-3-8B and the 1 GiB set, alternated, two rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_sched3; mkdir -p $O
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2; do
  b l_w128_$r X=1 -- --steps 8 --warmup 2
  b l_w64_$r X=1 -- --wave-mib 64 --streams 2 --steps 8 --warmup 2
  b l_w192_$r X=1 -- --wave-mib 192 --streams 2 --steps 8 --warmup 2
  b l_w256_$r X=1 -- --wave-mib 256 --streams 2 --steps 8 --warmup 2
  b l_up_$r OFL_EDEN_WAVESORT=2 -- --steps 8 --warmup 2
  b u_w128_$r X=1 -- --workload uniform_1gib --steps 30 --warmup 5
  b u_w64_$r X=1 -- --workload uniform_1gib --wave-mib 64 --streams 2 --steps 30 --warmup 5
  b u_w192_$r X=1 -- --workload uniform_1gib --wave-mib 192 --streams 2 --steps 30 --warmup 5
  b u_w256_$r X=1 -- --workload uniform_1gib --wave-mib 256 --streams 2 --steps 30 --warmup 5
done
