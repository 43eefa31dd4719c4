#!/bin/bash
# Round-5 closing bench lines with the per-workload stream defaults (GPU box, repo root): the default bench of every
# workload (CPU baseline included) and the bench-shape GPU tests.
set -e
O=gpurun_out/final10
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shape.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
head -c 300 $O/bench_default.json; echo
for W in extract stereo tracking; do
  timeout -k 10 500 python bench.py --workload $W > $O/bench_$W.json 2> $O/bench_$W.err || { tail -20 $O/bench_$W.err; exit 1; }
  head -c 200 $O/bench_$W.json; echo
done
echo final-f done
