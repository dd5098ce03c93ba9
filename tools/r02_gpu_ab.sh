#!/bin/bash
# Round-2 A/B call: GPU tests (Eden parity + lossy), the bench with the
# default build and with one env toggle, and a rocprof trace of the KC
# pipeline.  Usage (GPU box): bash tools/r02_gpu_ab.sh TAG ENVVAR=VALUE
set -euo pipefail
TAG=${1:-ab}; TOGGLE=${2:-OFL_EDEN_ROLL=0}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lossy.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
echo "pytest ok"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --also uniform_1gib > "$O/bench_default.json" 2> "$O/bench_default.err"
echo "bench default ok"
env "$TOGGLE" timeout -k 10 300 python -u bench.py --no-cpu-baseline --also uniform_1gib > "$O/bench_toggle.json" 2> "$O/bench_toggle.err"
echo "bench toggle ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_kc" -o run -- \
    python3 "$R/bench.py" --workload resnet50_fp32 --no-cpu-baseline --also kc_uniform_1gib --steps 5 \
    > "$R/$O/bench_kc_under_rocprof.json" 2> "$R/$O/prof_kc.err"
echo "rocprof kc ok"
