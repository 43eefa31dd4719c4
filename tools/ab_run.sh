set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_bench_shape.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_fast.log 2>&1 || { tail -30 gpurun_out/t_fast.log; exit 1; }
tail -2 gpurun_out/t_fast.log
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names nowl,wl; done
