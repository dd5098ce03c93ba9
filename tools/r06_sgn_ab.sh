#!/bin/bash
# r06: D1 sign bitmaps (k_signs) for the two-blocks-per-CU row kernels vs
# per-element hashing (OFL_EDEN_SGN=0): ResNet-50 and the 1 GiB set at MALL
# waves, no events; alternated, two rounds.  The Eden parity tests first.
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r06_sgn
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1
echo "parity rc=$?"; tail -n 2 $O/parity.log
for rep in 1 2; do
  for sg in 1 0; do
    OFL_EDEN_SGN=$sg timeout -k 10 200 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events \
        --workload resnet50_fp32 --steps 300 --warmup 20 > $O/rn_s${sg}_$rep.json 2> $O/rn_s${sg}_$rep.err || exit 3
    echo "rn sgn=$sg $rep $(python -c "import json;d=json.load(open('$O/rn_s${sg}_$rep.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"
    for w in 64 128; do
      OFL_EDEN_SGN=$sg OFL_EDEN_ROW2=1 timeout -k 10 200 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events \
        --workload uniform_1gib --wave-mib $w --streams 2 --steps 30 --warmup 5 > $O/u_s${sg}_w${w}_$rep.json 2> $O/u_s${sg}_w${w}_$rep.err || exit 2
      echo "u sgn=$sg w$w $rep $(python -c "import json;d=json.load(open('$O/u_s${sg}_w${w}_$rep.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"
    done
  done
done
