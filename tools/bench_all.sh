#!/bin/bash
# Every bench workload once (GPU box): config 3 (headline), config 2, config 4, config 5.  Each run has its own limit.
set -e
mkdir -p gpurun_out/all
for W in mono_init extract stereo tracking; do
  timeout -k 10 600 python bench.py --workload $W $BENCH_ARGS > gpurun_out/all/$W.json 2> gpurun_out/all/$W.err
  python -c "import json;d=json.load(open('gpurun_out/all/$W.json'));print('$W', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d.get('cpu_baseline') and d['cpu_baseline']['value'], d['stages_ms_per_launch'])"
done
