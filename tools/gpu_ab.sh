#!/bin/bash
# GPU box: the GPU test suite on the default build, then interleaved A/B rounds of experiment builds
# (tools/variant_bench.py).  AB_NAMES=a,b  AB_ROUNDS (default 3)  AB_EXTRA = extra bench args.  Each step has its
# own time limit and the script stops at the first failure.
set -e
OUT=gpurun_out/ab
mkdir -p $OUT
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 \
    || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
for i in $(seq 1 ${AB_ROUNDS:-3}); do
  timeout -k 10 300 python tools/variant_bench.py --streams ${AB_STREAMS:-2} --names ${AB_NAMES} -- --steps 30 ${AB_EXTRA:-} \
    | tee -a $OUT/ab.log
done
