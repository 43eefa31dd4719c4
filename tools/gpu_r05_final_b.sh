#!/bin/bash
# Round-5 final session B (GPU box, repo root): per workload PMC passes + per-stage summary (profiles/pmc_latest*.json),
# single-stream per-(kernel, batch) rocprof summary, and the default bench line reading the fresh PMC traffic
set -e
bash tools/gpu_r05_measure.sh mono_init extract stereo tracking > gpurun_out/meas_r05.log 2>&1 || { tail -20 gpurun_out/meas_r05.log; exit 1; }
tail -6 gpurun_out/meas_r05.log
