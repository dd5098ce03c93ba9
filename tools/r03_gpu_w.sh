#!/bin/bash
# Round 3, GPU call W: bytes_from recycling its own large payloads (default)
# vs off (OFL_HOST_RECYCLE=0): the -m gpu suite, the KC step statement by
# statement, the KC bench line, the e2e loopback.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3w
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 13
T 200 python -u tools/kc_gap.py > $O/gap_recycle.json 2> $O/gap_recycle.err || exit 11
T 200 env OFL_HOST_RECYCLE=0 python -u tools/kc_gap.py > $O/gap_off.json 2> $O/gap_off.err || exit 12
for rep in 1 2; do
  for v in "recycle" "off:OFL_HOST_RECYCLE=0"; do
    n=${v%%:*}; e=""; [ "$n" != "$v" ] && e=${v#*:}
    T 300 env $e python -u bench.py --workload uniform_1gib --steps 3 --warmup 1 --also kc_uniform_1gib --also-steps 20 --no-cpu-baseline > $O/kc_${rep}_$n.json 2> $O/kc_${rep}_$n.err || exit 14
  done
done
T 300 python -u tools/e2e_bench.py --modes plugin,batched --out $O/e2e_recycle.json > /dev/null 2> $O/e2e_recycle.err || exit 15
T 300 env OFL_HOST_RECYCLE=0 python -u tools/e2e_bench.py --modes plugin,batched --out $O/e2e_off.json > /dev/null 2> $O/e2e_off.err || exit 16
