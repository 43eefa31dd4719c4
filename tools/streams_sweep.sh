#!/bin/bash
# bench.py over 1/2/3/4 concurrent streams per GPU (GPU box; each run under its own limit)
set -e
mkdir -p gpurun_out/sweep
for S in ${STREAMS:-1 2 3 4}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --streams $S ${BENCH_EXTRA:-} > gpurun_out/sweep/s$S.json 2> gpurun_out/sweep/s$S.err
  python -c "import json;d=json.load(open('gpurun_out/sweep/s$S.json'));print($S, d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], d['stages_ms_per_launch'])"
done
