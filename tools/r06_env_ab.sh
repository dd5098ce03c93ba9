#!/bin/bash
# r06 A/B: HW queues (HIP default 4 vs 8) x NUMA binding, on bench.py's own
# process shape (Llama plan, the 1 GiB set with its graph capture, then KC),
# alternated, 3 rounds.  -> gpurun_out/r06_env_ab/*.json
set -o pipefail
out=gpurun_out/r06_env_ab; mkdir -p $out
for r in 1 2; do
  for cfg in q4_bind q4_free q8_bind q8_free; do
    a="--steps 3 --warmup 1 --also uniform_1gib,kc_uniform_1gib --no-cpu-baseline --also-steps 10"
    case $cfg in q8*) a="$a --hw-queues 8";; esac
    case $cfg in *bind) a="$a --numa-bind";; esac  # (the A/B ran when binding was the default and free took --no-numa-bind)
    timeout -k 10 240 python -u bench.py $a > $out/${cfg}_$r.json 2> $out/${cfg}_$r.err || exit 1
    python - $out/${cfg}_$r.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); k=d['also']['kc_uniform_1gib']
print(sys.argv[1], d['value'], d['also']['uniform_1gib']['value'], k['value'], k['phases_ms'], d['host_env'])
PY
  done
done
