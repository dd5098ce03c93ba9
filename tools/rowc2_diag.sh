#!/bin/bash
# k_enc_rowC2 cost breakdown: the Llama bench at --streams 1 (HIP events around
# every launch) with diagnostic builds that drop one part of the kernel each
# (tools/bin/libofl_diag<mask>.so, -DOFL_DIAG_ROWC2=<mask>: 1 = no F2
# exchanges, 2 = no quantiser, 4 = no dot reduction; wrong outputs).
set -e
O=${1:-gpurun_out/rowc2_diag}
mkdir -p "$O"
run() {  # name lib
    if [ -n "$2" ]; then export OFL_CODEC_LIB="$2"; else unset OFL_CODEC_LIB; fi
    timeout -k 10 240 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --also "" --streams 1 > "$O/$1.json" 2> "$O/$1.err"
    python - "$O/$1.json" "$1" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = {n: v for n, v in d["roofline"]["kernels"].items() if "rowC2" in n}
print(sys.argv[2], d["value"], {n: v["avg_us"] for n, v in k.items()}, flush=True)
PY
}
run default ""
for m in 1 2 4 7; do run diag$m "$PWD/tools/bin/libofl_diag$m.so"; done
