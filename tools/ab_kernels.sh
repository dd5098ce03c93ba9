#!/bin/bash
# A/B kernel variants on the GPU box: runs bench.py once per library and prints
# the per-kernel breakdown.  Usage: tools/ab_kernels.sh [lib.so ...]
# (the default build first; each run is time-limited on its own)
set -e
mkdir -p gpurun_out
run() {
  local tag=$1 lib=$2
  if [ -n "$lib" ]; then export OFL_CODEC_LIB=$lib; else unset OFL_CODEC_LIB; fi
  timeout -k 10 240 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err
  python - "$tag" <<'PY'
import json, sys
tag = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/ab_{tag}.json") if l.startswith("{")][-1])
print(f"== {tag}: {d['value']} GiB/s  {d['ms_per_step']} ms/step")
for k, v in d["roofline"]["kernels"].items():
    if v["share"] > 0.01:
        print(f"   {k:28s} {v['avg_us']:10.1f} us  {v['moved_GBps']:8.1f} GB/s")
PY
}
run base ""
for lib in "$@"; do run "$(basename $lib .so)" "$lib"; done
