#!/bin/bash
# A/B kernel variants on the GPU box: runs bench.py once per variant and prints
# the per-kernel breakdown.  Variants: a library path (*.so, via OFL_CODEC_LIB)
# or NAME=VALUE (an environment setting for that run).  The default build
# runs first.  Usage: tools/ab_kernels.sh [lib.so | VAR=value ...]
set -e
mkdir -p gpurun_out
run() {
  local tag=$1
  timeout -k 10 240 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --also "" ${AB_ARGS:-} > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err
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
run base
for v in "$@"; do
  if [[ "$v" == *.so ]]; then
    OFL_CODEC_LIB=$v run "$(basename $v .so)"
  else
    env $v bash -c "$(declare -f run); run '${v//[^A-Za-z0-9_]/_}'"
  fi
done
