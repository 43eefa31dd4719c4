#!/bin/bash
# round-4 GPU session 1: new parity tests, pyramid row-stream parity (ORBGPU_PYR_ROWS=1), then A/B timing
set -e
OUT=gpurun_out/s1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_binding_matchers.py tests/test_gpu_record.py tests/test_gpu_match.py \
  tests/test_gpu_projection.py -x -q --timeout 120 --timeout-method thread > $OUT/t_new.log 2>&1 || { tail -30 $OUT/t_new.log; exit 1; }
tail -1 $OUT/t_new.log
ORBGPU_PYR_ROWS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_semantics.py tests/test_gpu_bench_shape.py \
  -x -q --timeout 120 --timeout-method thread > $OUT/t_rows.log 2>&1 || { tail -30 $OUT/t_rows.log; exit 1; }
tail -1 $OUT/t_rows.log
for i in 1 2; do
  for v in 0 1; do
    ORBGPU_PYR_ROWS=$v timeout -k 10 200 python bench.py --steps 40 --no-cpu-baseline > $OUT/bench_rows$v.json 2> $OUT/bench_rows$v.err
    python -c "import json;d=json.load(open('$OUT/bench_rows$v.json'));print('rows$v', d['value'], d['parity']['mismatches'], {k:round(x,3) for k,x in d['stages_busy_ms_per_step'].items()})"
  done
done
AB_SKIP_TESTS=1 AB_NAMES=pk0,pk1 AB_ROUNDS=2 bash tools/gpu_ab.sh
