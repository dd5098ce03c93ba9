#!/bin/bash
# r06: nt (aux = 2) on the large slices' once-read / once-written arena I/O
# (x and plane loads: abvar/libofl_io_ld.so; y and plane stores: _st; both),
# so that at MALL-sized waves the streamed bytes do not push the wave's
# intermediates out of the Infinity Cache; vs the product library.  Parity
# subset with "both" first, then the Llama step and the 1 GiB set, x2.
# Variants: bash tools/build_flags_variant.sh abvar/libofl_io_{ld,st,both}.so -DOFL_IO_{LD,ST}_AUX=2
set -uo pipefail
R=$PWD; O=$R/gpurun_out/r06_io_nt; mkdir -p $O
OFL_CODEC_LIB=$R/abvar/libofl_io_both.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "five_pass or schedules or row2 or golden or oracle or wavg" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 11
b() { local tag=$1; shift; local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --also "" --no-cpu-baseline --no-kernel-events "$@" > $O/$tag.json 2>/dev/null || exit 2
  echo "$tag $(python -c "import json;d=json.load(open('$O/$tag.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"; }
for r in 1 2; do
  for v in prod ld st both; do
    if [ $v = prod ]; then e=X=1; else e=OFL_CODEC_LIB=$R/abvar/libofl_io_$v.so; fi
    b l_${v}_$r $e -- --steps 8 --warmup 2
    b u_${v}_$r $e -- --workload uniform_1gib --steps 30 --warmup 5
  done
done
