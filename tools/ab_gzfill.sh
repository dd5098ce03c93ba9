# A/B of the KC step: in-tree library (payload filled during the encode) and
# build/var/*.so variants; tools/kc_step_probe.py splits the host side
set -e
mkdir -p gpurun_out/gzfill
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lossy.py -k "gzip" > gpurun_out/gzfill/pytest.log 2>&1
for v in base c12s4; do
  if [ $v = base ]; then L=$PWD/openfl_amd/lib/libofl_codec.so; else L=$PWD/build/var/$v.so; fi
  OFL_CODEC_LIB=$L timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 > gpurun_out/gzfill/kc_$v.json 2> gpurun_out/gzfill/kc_$v.err
  OFL_CODEC_LIB=$L timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 > gpurun_out/gzfill/kc2_$v.json 2> gpurun_out/gzfill/kc2_$v.err
done
timeout -k 10 150 python -u tools/kc_step_probe.py --steps 8 > gpurun_out/gzfill/probe.json 2> gpurun_out/gzfill/probe.err
