#!/bin/bash
# Round 3, GPU call T: the final tree's health -- the whole -m gpu suite,
# smoke(), the default bench line (as the driver runs it).  gpurun_out/r3t/.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r3t
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 13
T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 14
T 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 15
