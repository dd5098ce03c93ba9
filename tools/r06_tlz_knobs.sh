#!/bin/bash
# r06 TLZ encoder candidates x DP sweeps (library variants, tools/build_flags_variant.sh
# -DOFL_TLZ_CAND / -DOFL_TLZ_SWEEPS): KC steps (tools/kc_bench.py, NUMA-bound) and
# the wire ratio, alternated, three rounds.  c11s4 = the product.
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_tlz_knobs; mkdir -p $O
for r in 1 2 3; do
  for v in c11s4 c11s3 c10s4 c10s3; do
    lib=$R/tools/bin/tlz/$v.so; [ $v = c11s4 ] && lib=$R/openfl_amd/lib/libofl_codec.so
    OFL_CODEC_LIB=$lib timeout -k 10 200 python -u tools/kc_bench.py --steps 10 --warmup 3 > $O/${v}_$r.json 2> $O/${v}_$r.err || exit 2
    echo "$v $r $(python -c "import json;d=json.load(open('$O/${v}_$r.json'));print(d['value'],d['ms_per_step'],d['wire_ratio'],d['phases_ms'])")"
  done
done
