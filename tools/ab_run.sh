#!/bin/bash
# GPU box: full GPU test suite on the default build, then interleaved A/B of two experiment builds
# (tools/variant_bench.py; AB_NAMES=a,b; AB_EXTRA = extra bench args)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -2 gpurun_out/t_all.log
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names ${AB_NAMES} -- ${AB_EXTRA:-}; done
