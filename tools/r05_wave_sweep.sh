#!/bin/bash
# Round 5: MALL-sized waves in the real codec (tools/dataflow_bench.hip showed
# per-pass launches over 64-128 MiB waves moving the codec's bytes at 6.4-7.0
# TB/s against 4.5-5.4 TB/s over 2 GiB waves).  bench.py lines per schedule,
# Llama-3-8B and the 1 GiB set; OFL_EDEN_ROW2=1 forces the two-blocks-per-CU
# row kernels.  Outputs: gpurun_out/$1/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/${1:-r05c}
mkdir -p $O
T() { timeout -k 10 "$@"; }
run() {  # tag workload wave streams row2
  local tag=$1 wl=$2 w=$3 s=$4 r2=$5
  OFL_EDEN_ROW2=$r2 T 200 python -u bench.py --workload $wl --also "" --no-cpu-baseline --wave-mib $w --streams $s \
      --steps 10 --warmup 3 > $O/$tag.json 2> $O/$tag.err
  local rc=$?
  echo "$tag rc=$rc $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('dominant_kernel',{}).get('name'))" 2>/dev/null)" >> $O/summary.txt
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && exit 20
  return 0
}
run u_w2048_s1 uniform_1gib 2048 1 ""
run u_w64_s1_r2 uniform_1gib 64 1 1
run u_w128_s1_r2 uniform_1gib 128 1 1
run u_w64_s2_r2 uniform_1gib 64 2 1
run u_w128_s2_r2 uniform_1gib 128 2 1
run l_w2048_s2 llama3_8b_fp32_update 2048 2 ""
run l_w128_s1_r2 llama3_8b_fp32_update 128 1 1
run l_w128_s2_r2 llama3_8b_fp32_update 128 2 1
run l_w256_s1_r2 llama3_8b_fp32_update 256 1 1
run l_w64_s2_r2 llama3_8b_fp32_update 64 2 1
run l_w128_s1 llama3_8b_fp32_update 128 1 ""
echo "sweep done" >> $O/summary.txt
