#!/bin/bash
# Round-4 final measurement session (GPU box, repo root): GPU suite, then per workload PMC + per-batch kernel
# summary + default bench (tools/gpu_r04_measure.sh), then the headline bench line with its CPU baseline and the
# FAST phase profile.  Every GPU step has its own time limit; the script stops at the first failure.
set -e
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final/tests.log 2>&1 \
  || { tail -30 gpurun_out/final/tests.log; exit 1; }
tail -1 gpurun_out/final/tests.log
bash tools/gpu_r04_measure.sh mono_init tracking stereo extract > gpurun_out/final/measure.log 2>&1 || { tail -20 gpurun_out/final/measure.log; exit 1; }
tail -5 gpurun_out/final/measure.log
timeout -k 10 400 python bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err
head -c 400 gpurun_out/final/bench_default.json; echo
timeout -k 10 200 python tools/fast_profile.py --run --batch 256 > gpurun_out/final/fast_profile.txt 2>&1 || true
