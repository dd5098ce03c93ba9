#!/bin/bash
# Does Infinity-Cache residency speed the large-slice passes up?  Per-kernel
# HIP-event averages (one stream) and PMC traffic of the 1 GiB set with waves
# whose intermediates fit the 256 MiB cache (64 / 128 MiB) vs 2 GiB waves.
# Usage (GPU box, repo root): bash tools/mall_kernel_ab.sh TAG
set -euo pipefail
TAG=${1:-mall}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/$TAG
mkdir -p "$R/$O"
for m in 2048 128 64; do
  timeout -k 10 120 python -u bench.py --workload uniform_1gib --also "" --no-cpu-baseline --streams 1 \
      --wave-mib $m --steps 20 --warmup 3 > "$R/$O/bench_w$m.json" 2> "$R/$O/bench_w$m.err"
  echo "events w$m done"
  PMC_PASSES=traffic timeout -k 10 300 bash tools/pmc_run.sh "$O/pmc_w$m" --workload uniform_1gib --also "" \
      --streams 1 --wave-mib $m --steps 5 --warmup 2
  python tools/pmc_traffic.py "$R/$O/pmc_w$m" 7 "$R/$O/traffic_w$m.json" > /dev/null
  echo "pmc w$m done"
done
