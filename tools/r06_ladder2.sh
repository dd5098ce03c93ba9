#!/bin/bash
# r06 ladder, part 2: step times WITHOUT per-launch events in the timed
# region (bench.py --no-kernel-events; at 64 MiB waves a step has 112
# launches), one and two streams, rungs lad1 and full; rocprofv3 kernel
# durations of the same at 64 MiB waves; the memory-only microbenchmark
# (tools/dataflow_bench.hip) beside them; then the narrow-intermediate stubs
# (OFL_WS_FMT=16 / 24) against the product on the Llama step, alternated.
# Outputs: gpurun_out/r06_ladder2/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r06_ladder2
mkdir -p $O
T() { timeout -k 10 "$@"; }
lib() { case $1 in full) echo $R/openfl_amd/lib/libofl_codec.so;; *) echo $R/tools/bin/lad/libofl_$1.so;; esac; }
for l in lad1 full; do
  for s in 1 2; do
    for w in 64 128 2048; do
      r2=1; [ $w = 2048 ] && r2=""
      OFL_CODEC_LIB=$(lib $l) OFL_EDEN_ROW2=$r2 T 200 python -u bench.py --workload uniform_1gib --also "" \
          --no-cpu-baseline --no-kernel-events --wave-mib $w --streams $s --steps 20 --warmup 3 > $O/${l}_s${s}_w$w.json 2> $O/${l}_s${s}_w$w.err || exit 2
      echo "$l s$s w$w $(python -c "import json;d=json.load(open('$O/${l}_s${s}_w$w.json'));print(d['value'],d['ms_per_step'],d['gpu_ms_per_step_rank0'])")"
    done
  done
done
T 300 tools/bin/dataflow_bench 30 5 > $O/dataflow_bench.txt 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
for l in lad1 full; do
  OFL_CODEC_LIB=$(lib $l) OFL_EDEN_ROW2=1 T 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${l}_w64 -o run -- \
      python3 $R/bench.py --workload uniform_1gib --also "" --no-cpu-baseline --no-kernel-events --wave-mib 64 \
      --streams 1 --steps 5 --warmup 2 > $O/prof_${l}_w64.json 2> $O/prof_${l}_w64.err || exit 4
done
cd $R
for r in 1 2; do
  for l in full ws16 ws24; do
    OFL_CODEC_LIB=$(lib $l) T 300 python -u bench.py --also "" --no-cpu-baseline --steps 10 --warmup 3 > $O/llama_${l}_$r.json 2> $O/llama_${l}_$r.err || exit 5
    echo "llama $l $r $(python -c "import json;d=json.load(open('$O/llama_${l}_$r.json'));print(d['value'],d['ms_per_step'],d['check_rel_l2'],[(k,v['avg_us']) for k,v in list(d['roofline']['kernels'].items())[:6]])")"
  done
done
echo "ladder2 done"
