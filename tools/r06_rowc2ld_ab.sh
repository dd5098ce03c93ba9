#!/bin/bash
# r06: k_enc_rowC2's intermediate loads (the encode's last read of a wave's
# ws) nt (the product, OFL_ROWC2_LD_AUX=2 since round 3) vs the default policy
# (abvar/libofl_rowc2ld0.so) now that the arena I/O is nt: Llama-3-8B and the
# 1 GiB set, alternated x3.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_rowc2ld; mkdir -p $O
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2 3; do
  for v in prod rowc2ld0; do
    if [ $v = prod ]; then e=X=1; else e=OFL_CODEC_LIB=$R/abvar/libofl_$v.so; fi
    b l_${v}_$r $e -- --steps 8 --warmup 2
    b u_${v}_$r $e -- --workload uniform_1gib --steps 30 --warmup 5
  done
done
