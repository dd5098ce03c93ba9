#!/bin/bash
# Round 5, GPU call d: TLZ encoder DP / bit-emission rework and the batch
# loop without the side-stream scan: lossy GPU tests, A/B of the streams
# (must be byte-identical) and times against the previous build, the KC line.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r05d
mkdir -p $O
T() { timeout -k 10 "$@"; }
T 400 python -u -m pytest tests/test_gpu_lossy.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lossy.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_lossy.log
[ $rc -eq 0 ] || exit 11
OFL_CODEC_LIB=tools/bin/var/libofl_codec_gzbase.so T 200 python -u tools/tlz_ab.py base > $O/ab.jsonl 2> $O/ab_base.err || exit 12
T 200 python -u tools/tlz_ab.py new >> $O/ab.jsonl 2> $O/ab_new.err || exit 13
OFL_CODEC_LIB=tools/bin/var/libofl_codec_gzbase.so T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_base.json 2> $O/kc_base.err || exit 14
T 300 python -u tools/kc_bench.py --steps 10 --warmup 2 > $O/kc_new.json 2> $O/kc_new.err || exit 15
OFL_GZ_PHASES=1 T 120 python -u tools/tlz_phases.py > $O/tlz_phases.txt 2>&1 || exit 16
OFL_GZ_FILL_TRACE=1 T 200 python -u tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_trace.json 2> $O/kc_fill_trace.txt || exit 17
cd /tmp && export TMPDIR=/tmp
T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kc_trace -o k -- python3 $R/tools/kc_bench.py --steps 3 --warmup 1 > $O/kc_rocprof.log 2>&1 || exit 24
echo "r05d done"
