#!/bin/bash
# Round 5 session 3: A/B of FAST's one-reservation-per-wave stage 1 (OG_FASTQ_WAT) and the two-/four-tile pipelined
# fused resize (RZ2_TPW) against the committed build (base): headline bench lines (each with its parity check), then
# single-stream rocprof per-kernel times of each library, then the extraction parity tests of the default build
set -e
mkdir -p gpurun_out/r05
for i in 1 2; do timeout -k 10 400 python tools/variant_bench.py --streams 2 --names base,f1r1,f0r1,f1r2,f1r2w5,f1r4 -- --steps 100; done > gpurun_out/r05/ab3_mono.log 2>&1 || { tail -20 gpurun_out/r05/ab3_mono.log; exit 1; }
cat gpurun_out/r05/ab3_mono.log
for v in base f1r1 f0r1 f1r2 f1r4; do ORBGPU_LIB=$PWD/orbslam2_with_quadrics_amd/variants/liborbgpu_$v.so bash tools/gpu_kstats.sh ab3_$v mono_init > gpurun_out/r05/ks_ab3_$v.log 2>&1; echo "== $v"; grep -E "fast_quad|resize2|resize_kernel" gpurun_out/r05/ks_ab3_$v.log | grep "| 512 |"; done
timeout -k 10 500 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_bench_shape.py tests/test_gpu_semantics.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/t_s3.log 2>&1 || { tail -40 gpurun_out/r05/t_s3.log; exit 1; }
tail -2 gpurun_out/r05/t_s3.log
