#!/bin/bash
# r06: the additive LCG in the two-blocks-per-CU row kernels' D1 signs
# (p >= 18: one quarter-rate multiply per element fewer) vs the previous
# library (tools/bin/lad/libofl_prev.so): Eden parity tests, then ResNet-50,
# the 1 GiB set at 128 MiB waves (two streams) and the default Llama step,
# alternated, three rounds.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_lcg; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -n 2 $O/parity.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for v in new prev; do
    lib=$R/openfl_amd/lib/libofl_codec.so; [ $v = prev ] && lib=$R/tools/bin/lad/libofl_prev.so
    OFL_CODEC_LIB=$lib timeout -k 10 200 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events --workload resnet50_fp32 --steps 300 --warmup 20 > $O/rn_${v}_$r.json 2>/dev/null || exit 2
    OFL_CODEC_LIB=$lib OFL_EDEN_ROW2=1 timeout -k 10 200 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events --workload uniform_1gib --wave-mib 128 --streams 2 --steps 30 --warmup 5 > $O/u_${v}_$r.json 2>/dev/null || exit 3
    echo "$v $r rn $(python -c "import json;d=json.load(open('$O/rn_${v}_$r.json'));print(d['value'],d['gpu_ms_per_step_rank0'])") u128 $(python -c "import json;d=json.load(open('$O/u_${v}_$r.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"
  done
done
