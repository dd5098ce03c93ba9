set -e
mkdir -p gpurun_out/cand
for v in c16s4 c14s4 c12s4 c10s4; do
  if [ $v = c16s4 ]; then L=$PWD/openfl_amd/lib/libofl_codec.so; else L=$PWD/build/var/$v.so; fi
  echo "== $v" | tee -a gpurun_out/cand/ab.txt
  OFL_CODEC_LIB=$L timeout -k 10 150 python -u tools/tlz_check.py --big >> gpurun_out/cand/ab.txt 2>&1
  OFL_CODEC_LIB=$L timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 > gpurun_out/cand/kc_$v.json 2> gpurun_out/cand/kc_$v.err
  tail -c 400 gpurun_out/cand/kc_$v.json
done
