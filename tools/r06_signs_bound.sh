#!/bin/bash
# r06: the bound of cheaper sign generation at MALL waves: the product with
# the D1 / D2 sign work compiled out (-DOFL_LADDER=5, wrong results) against
# the product, 1 GiB set and ResNet-50, two streams, no events.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r06_signs
mkdir -p $O
for rep in 1 2; do
  for l in full lad5; do
    lib=$R/openfl_amd/lib/libofl_codec.so; [ $l = lad5 ] && lib=$R/tools/bin/lad/libofl_lad5.so
    for w in 64 128; do
      OFL_CODEC_LIB=$lib OFL_EDEN_ROW2=1 timeout -k 10 200 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events \
        --workload uniform_1gib --wave-mib $w --streams 2 --steps 30 --warmup 5 > $O/u_${l}_w${w}_$rep.json 2> $O/u_${l}_w${w}_$rep.err || exit 2
      echo "u $l w$w $rep $(python -c "import json;d=json.load(open('$O/u_${l}_w${w}_$rep.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"
    done
    OFL_CODEC_LIB=$lib timeout -k 10 200 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events \
        --workload resnet50_fp32 --steps 300 --warmup 20 > $O/rn_${l}_$rep.json 2> $O/rn_${l}_$rep.err || exit 3
    echo "rn $l $rep $(python -c "import json;d=json.load(open('$O/rn_${l}_$rep.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"
  done
done
