#!/bin/bash
# r06 ladder: the real large-slice kernels with their
# work added back one rung at a time (-DOFL_LADDER, eden_kernels.hip; wrong
# results, diagnostics only): 1 = tile loads/stores only, 2 = + butterflies
# and LDS exchanges, 3 = + sign generation, full = + quantiser / unpack /
# reductions (the product library).  The 1 GiB set (64 x 2^22 slices), one
# stream, the two-blocks-per-CU row kernels at 64 / 128 MiB waves and the
# default kernels at one 1 GiB wave; per-kernel HIP events inside the timed
# region; then rocprofv3 SQ counter passes per rung at 64 MiB waves.
# Outputs: gpurun_out/r06_ladder/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r06_ladder
mkdir -p $O
T() { timeout -k 10 "$@"; }
lib() { case $1 in full) echo $R/openfl_amd/lib/libofl_codec.so;; *) echo $R/tools/bin/lad/libofl_$1.so;; esac; }
for l in lad1 lad2 lad3 full; do
  for w in 64 128 2048; do
    r2=1; [ $w = 2048 ] && r2=""
    OFL_CODEC_LIB=$(lib $l) OFL_EDEN_ROW2=$r2 T 200 python -u bench.py --workload uniform_1gib --also "" \
        --no-cpu-baseline --wave-mib $w --streams 1 --steps 10 --warmup 3 > $O/${l}_w$w.json 2> $O/${l}_w$w.err || exit 2
    echo "$l w$w $(python -c "import json;d=json.load(open('$O/${l}_w$w.json'));print(d['value'],d['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
for l in lad1 lad2 lad3 full; do
  i=0
  for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    OFL_CODEC_LIB=$(lib $l) OFL_EDEN_ROW2=1 T 120 rocprofv3 --pmc $pmc --output-format csv -d $O/sq_${l}_w64/pass$i -o p -- \
        python3 $R/bench.py --workload uniform_1gib --also "" --no-cpu-baseline --no-kernel-events --wave-mib 64 \
        --streams 1 --steps 3 --warmup 1 > $O/sq_${l}_$i.log 2>&1 || exit 3
  done
  (cd $R && python tools/pmc_kernels.py $O/sq_${l}_w64 $O/sq_${l}_w64.json k_enc k_dec k_col > /dev/null) || exit 4
  echo "sq $l done"
done
echo "ladder done"
