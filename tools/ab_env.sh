#!/bin/bash
# A/B of one library env toggle on a workload: bash tools/ab_env.sh VAR WORKLOAD [runs]
set -e
VAR=$1; WL=$2; N=${3:-3}
B=(python bench.py --workload "$WL" --no-cpu-baseline --also= --steps 100 --warmup 5 --no-kernel-events)
for i in $(seq "$N"); do
  echo "on  $(timeout -k 10 120 "${B[@]}" 2>/dev/null | grep -o '"value": [0-9.]*')"
  echo "off $(env "$VAR=0" timeout -k 10 120 "${B[@]}" 2>/dev/null | grep -o '"value": [0-9.]*')"
done
