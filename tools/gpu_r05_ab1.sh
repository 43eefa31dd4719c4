#!/bin/bash
# Round 5: wave-per-cell FAST (og_fast_cell_kernel) -- parity on the extraction/matcher tests, A/B vs the block
# kernel (variants/liborbgpu_{quad,cell}.so), single-stream rocprof summary, then the whole GPU suite
set -e
mkdir -p gpurun_out/r05
timeout -k 10 500 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_bench_shape.py tests/test_gpu_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/t_ext.log 2>&1 || { tail -40 gpurun_out/r05/t_ext.log; exit 1; }
tail -2 gpurun_out/r05/t_ext.log
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names quad,cell -- --steps 100; done > gpurun_out/r05/ab_mono.log 2>&1
cat gpurun_out/r05/ab_mono.log
timeout -k 10 300 python tools/variant_bench.py --streams 2 --names quad,cell -- --workload stereo --steps 100 > gpurun_out/r05/ab_stereo.log 2>&1
cat gpurun_out/r05/ab_stereo.log
bash tools/gpu_kstats.sh cell mono_init > gpurun_out/r05/ks_cell.log 2>&1 && head -14 gpurun_out/r05/ks_cell.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/t_all.log 2>&1 || { tail -40 gpurun_out/r05/t_all.log; exit 1; }
tail -2 gpurun_out/r05/t_all.log
