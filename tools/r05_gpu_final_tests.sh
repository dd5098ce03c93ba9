#!/bin/bash
# Round 5: the -m gpu suite on the current tree, then smoke().
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05ft2
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 11
T 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 12

T 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 13
echo "bench done"
