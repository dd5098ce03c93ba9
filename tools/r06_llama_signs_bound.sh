set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_l5; mkdir -p $O
for rep in 1 2; do
 for l in full lad5; do
  lib=$R/openfl_amd/lib/libofl_codec.so; [ $l = lad5 ] && lib=$R/tools/bin/lad/libofl_lad5.so
  for w in 128 2048; do
    r2=1; [ $w = 2048 ] && r2=""
    OFL_CODEC_LIB=$lib OFL_EDEN_ROW2=$r2 timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events --wave-mib $w --streams 2 --steps 8 --warmup 2 > $O/l_${l}_w${w}_$rep.json 2> $O/l_${l}_w${w}_$rep.err || exit 2
    echo "llama $l w$w $rep $(python -c "import json;d=json.load(open('$O/l_${l}_w${w}_$rep.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"
  done
 done
done
