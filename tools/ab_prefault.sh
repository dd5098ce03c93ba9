# KC step with and without the payload prefault (OFL_GZ_NO_PREFAULT=1), one box
set -e
mkdir -p gpurun_out/pfab
for r in 1 2 3; do
  OFL_GZ_FILL_TRACE=1 timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 >> gpurun_out/pfab/kc_pf.json 2>> gpurun_out/pfab/kc_pf.err
  OFL_GZ_NO_PREFAULT=1 OFL_GZ_FILL_TRACE=1 timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 >> gpurun_out/pfab/kc_nopf.json 2>> gpurun_out/pfab/kc_nopf.err
done
