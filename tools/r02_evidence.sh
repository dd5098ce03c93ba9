#!/bin/bash
# Round-2 evidence for the headline bench line, in one GPU call (repo root on
# the GPU box):  bash tools/r02_evidence.sh TAG
#   1. PMC HBM traffic of the default Llama-3-8B bench (FETCH_SIZE / WRITE_SIZE
#      passes, tools/pmc_run.sh + pmc_traffic.py)
#   2. the default bench line with that traffic attached
#   3. rocprofv3 --kernel-trace --stats of the default schedule and of --streams 1
#   4. PMC traffic of the KC pipeline kernels (lossy:: k-means/LUT, gz:: gzip)
# Outputs under gpurun_out/evidence_TAG/.
set -euo pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=gpurun_out/evidence_$TAG
mkdir -p "$R/$O"
cd "$R"
PMC_PASSES=traffic timeout -k 10 600 bash tools/pmc_run.sh "$O/pmc" --steps 5 --warmup 2 --also ""
python tools/pmc_traffic.py "$R/$O/pmc" 7 "$R/$O/hbm_traffic.json" > /dev/null
echo "pmc done"
timeout -k 10 600 python -u bench.py --traffic-json "$R/$O/hbm_traffic.json" > "$R/$O/bench.json" 2> "$R/$O/bench.err"
echo "bench done"
PMC_PASSES=traffic timeout -k 10 600 bash tools/pmc_run.sh "$O/pmc_kc" --workload mnist_cnn --also kc_uniform_1gib --steps 2 --warmup 1
python tools/pmc_traffic.py "$R/$O/pmc_kc" 3 "$R/$O/kc_traffic.json" > /dev/null
echo "pmc kc done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_default" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --also "" > "$R/$O/bench_default_under_rocprof.json" 2> "$R/$O/prof_default.err"
echo "rocprof default done"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_1stream" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --also "" --streams 1 > "$R/$O/bench_1stream_under_rocprof.json" 2> "$R/$O/prof_1stream.err"
echo "rocprof 1-stream done"
