#!/bin/bash
# r06 KC decode knobs: staged-H2D threads (OFL_H2D_THREADS) x inflate pieces
# (OFL_INFLATE_PIECES), tools/kc_bench.py --steps 10 --warmup 3 (NUMA-bound),
# alternated, three rounds.  Outputs: gpurun_out/r06_kc_knobs/
set -uo pipefail
O=$PWD/gpurun_out/r06_kc_knobs; mkdir -p $O
for r in 1 2 3; do
  for th in 2 4; do
    for pc in 4 8; do
      OFL_H2D_THREADS=$th OFL_INFLATE_PIECES=$pc timeout -k 10 200 python -u tools/kc_bench.py --steps 10 --warmup 3 > $O/t${th}_p${pc}_$r.json 2> $O/t${th}_p${pc}_$r.err || exit 2
      echo "t$th p$pc $r $(python -c "import json;d=json.load(open('$O/t${th}_p${pc}_$r.json'));print(d['value'],d['ms_per_step'],d['phases_ms'])")"
    done
  done
done
