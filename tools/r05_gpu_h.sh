#!/bin/bash
# Round 5, GPU call h: pipelined inflate piece count, alternated (noise).
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05h
mkdir -p $O
T() { timeout -k 10 "$@"; }
for r in 1 2 3; do
for p in 1 2 3 4; do
  OFL_INFLATE_PIECES=$p T 300 python -u tools/kc_bench.py --steps 15 --warmup 3 > $O/kc_p${p}_$r.json 2> $O/kc_p${p}_$r.err || exit 15
  python -c "import json;d=json.load(open('$O/kc_p${p}_$r.json'));print('pieces=$p',d['value'],d['ms_per_step'],d['phases_ms'],d['wire_ratio'])" >> $O/summary.txt
done
done
echo "r05h done"
