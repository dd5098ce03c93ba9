#!/bin/bash
# r06: the Llama line's two modes (~425 vs ~437 GiB/s): repeated default runs
# and two kernel traces.  Outputs: gpurun_out/r06_modes/
set -uo pipefail
R=$PWD
O=$R/gpurun_out/r06_modes
mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 200 python -u bench.py --also "" --no-cpu-baseline --steps 10 --warmup 3 > $O/b$i.json 2> $O/b$i.err || exit 2
  echo "b$i $(python -c "import json;d=json.load(open('$O/b$i.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"
done
cd /tmp && export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace$i -o t -- python3 $R/bench.py --also "" --no-cpu-baseline --no-kernel-events --steps 6 --warmup 2 > $O/t$i.json 2> $O/t$i.err || exit 3
  echo "t$i $(python3 -c "import json;d=json.load(open('$O/t$i.json'));print(d['value'],d['gpu_ms_per_step_rank0'])")"
done
