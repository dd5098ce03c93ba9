# KC step vs the inflate's staging threads (OFL_H2D_THREADS)
set -e
mkdir -p gpurun_out/h2dt
for t in 2 3 4 1 2 3 4; do
  OFL_H2D_THREADS=$t timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 >> gpurun_out/h2dt/kc_$t.json 2>> gpurun_out/h2dt/kc_$t.err
done
