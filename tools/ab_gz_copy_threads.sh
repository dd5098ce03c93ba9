# KC step vs the gzip payload fill threads (OFL_GZ_COPY_THREADS), traced
set -e
mkdir -p gpurun_out/gzct
for t in 8 16 4 8 16 4; do
  OFL_GZ_COPY_THREADS=$t OFL_GZ_FILL_TRACE=1 timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 >> gpurun_out/gzct/kc_$t.json 2>> gpurun_out/gzct/kc_$t.err
done
