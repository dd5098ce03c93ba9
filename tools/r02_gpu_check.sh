#!/bin/bash
# Round-2 GPU check: the whole -m gpu suite, then the default bench line.
# Usage (GPU box, repo root): bash tools/r02_gpu_check.sh TAG
set -euo pipefail
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$O/pytest_gpu.log" 2>&1
echo "pytest ok"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
echo "bench ok"
