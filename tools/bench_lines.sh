#!/bin/bash
# Default bench line of each workload (GPU box): gpurun_out/lines/bench_<workload>.json.  traffic comes from the
# committed PMC files (profiles/pmc_latest[_<workload>].json), as in tools/gpu_measure_all.sh.
set -e
mkdir -p gpurun_out/lines
for W in ${@:-mono_init extract stereo tracking}; do
  timeout -k 10 400 python3 bench.py --workload $W > gpurun_out/lines/bench_$W.json 2> gpurun_out/lines/bench_$W.err
  echo "$W $(head -c 200 gpurun_out/lines/bench_$W.json)"
done
