#!/bin/bash
# Quick GPU iteration: parity tests + one default bench line (each step under its own time limit).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
cat gpurun_out/bench_quick.json
