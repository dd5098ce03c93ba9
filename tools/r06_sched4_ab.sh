#!/bin/bash
# r06: wave size again with nt arena I/O (the streamed bytes no longer
# compete with the intermediates for the MALL): 128 (default) vs 96 / 192 /
# 256 MiB on two streams, Llama-3-8B and the 1 GiB set, alternated x2.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_sched4; mkdir -p $O
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2; do
  for w in 128 96 192 256; do
    b l_w${w}_$r X=1 -- --wave-mib $w --streams 2 --steps 8 --warmup 2
    b u_w${w}_$r X=1 -- --workload uniform_1gib --wave-mib $w --streams 2 --steps 30 --warmup 5
  done
done
