#!/bin/bash
# Round 5, GPU call ab: the gzip side stream's HW queue -- 3 streams made
# first (the side stream then shares the caller's queue), with the default
# 4 HW queues, with 8, and with a high-priority side stream.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05ab
mkdir -p $O
T() { timeout -k 10 "$@"; }
for r in 1 2; do
  T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --extra-streams 3 > $O/kc_q4_$r.json 2> $O/kc_q4_$r.err || exit 11
  GPU_MAX_HW_QUEUES=8 T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --extra-streams 3 > $O/kc_q8_$r.json 2> $O/kc_q8_$r.err || exit 12
  OFL_GZ_SIDE_PRIO=1 T 300 python -u tools/kc_bench.py --steps 10 --warmup 4 --extra-streams 3 > $O/kc_prio_$r.json 2> $O/kc_prio_$r.err || exit 13
done
echo "r05ab done"
