# KC step with the host fill traced (OFL_GZ_FILL_TRACE=1), the in-tree
# library (12 candidates) and build/var/c16s4.so; the gzip GPU tests first
set -e
mkdir -p gpurun_out/fill2
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lossy.py -k "gzip or tlz or inflate" > gpurun_out/fill2/pytest.log 2>&1
OFL_GZ_FILL_TRACE=1 timeout -k 10 150 python -u tools/kc_bench.py --steps 6 --warmup 2 > gpurun_out/fill2/kc.json 2> gpurun_out/fill2/kc.err
OFL_CODEC_LIB=$PWD/build/var/c16s4.so timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 > gpurun_out/fill2/kc_c16.json 2> gpurun_out/fill2/kc_c16.err
timeout -k 10 150 python -u tools/kc_bench.py --steps 10 --warmup 2 > gpurun_out/fill2/kc_c12.json 2> gpurun_out/fill2/kc_c12.err
timeout -k 10 150 python -u tools/tlz_check.py --big > gpurun_out/fill2/tlz_c12.txt 2>&1
