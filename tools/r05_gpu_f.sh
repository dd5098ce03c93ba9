#!/bin/bash
# Round 5, GPU call f: KC line with the pooled host copies, and the TLZ
# encoder's candidate / sweep count A/B (ratio vs time).  Outputs gpurun_out/r05f/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05f
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_new.json 2> $O/kc_new.err || exit 15
OFL_GZ_FILL_TRACE=1 T 200 python -u tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.json 2> $O/kc_fill_trace.txt || exit 17
for v in c10 c11 s3; do
  OFL_CODEC_LIB=tools/bin/var/libofl_$v.so T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_$v.json 2> $O/kc_$v.err || exit 18
done
T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_new2.json 2> $O/kc_new2.err || exit 19
echo "r05f done"
