# payload filled during the encode (OFL_GZ_FILL=1, default) vs copied after (0)
set -e
mkdir -p gpurun_out/fill3
for f in 0 1 0 1; do
  OFL_GZ_FILL=$f timeout -k 10 150 python -u tools/tlz_check.py --big > gpurun_out/fill3/tlz_$f.txt 2>&1
  OFL_GZ_FILL=$f timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 >> gpurun_out/fill3/kc_$f.json 2>> gpurun_out/fill3/kc_$f.err
done
