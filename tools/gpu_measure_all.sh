#!/bin/bash
# Measurement session for the given bench workloads (GPU box, repo root), default all four:
#   1. PMC passes (tools/pmc_profile.sh) -> per-stage summary -> profiles/pmc_latest[_<workload>].json (box copy)
#   2. rocprofv3 --kernel-trace --stats of a single-stream run (launches do not overlap: per-kernel durations),
#      summarised per (kernel, frames per launch) by tools/prof_summary.py
#   3. the default bench run of the workload (reads the fresh PMC file for roofline.traffic)
# The PMC summary's frames per launch follow bench.py's defaults (512 frames over DEFAULT_STREAMS contexts).
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
OUT=${MEAS_OUT:-gpurun_out/meas}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
WORKLOADS=${@:-mono_init extract stereo tracking}
for W in $WORKLOADS; do
  P=$([ "$W" = mono_init ] && echo pmc_latest || echo pmc_latest_$W)
  B=$(python3 -c "import bench; print(512 // bench.DEFAULT_STREAMS['$W'])")
  timeout -k 10 400 bash tools/pmc_profile.sh "$OUT/pmc_$W" --workload $W --steps 3 --warmup 1 --no-cpu-baseline
  python3 tools/pmc_summary.py "$OUT/pmc_$W" --json "$OUT/$P.json" --md "$OUT/pmc_summary_$W.md" --batch $B
  cp "$OUT/$P.json" "profiles/$P.json"
  echo "$W: pmc done"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof_$W" -o run \
      -- python3 "$ROOT/bench.py" --workload $W --streams 1 --steps 20 --warmup 2 --no-cpu-baseline \
      > "$ROOT/$OUT/bench_${W}_streams1_rocprof.json" 2> "$ROOT/$OUT/rocprof_$W.err")
  find "$OUT/prof_$W" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_$W.csv" \;
  T=$(find "$OUT/prof_$W" -name "*kernel_trace.csv" | head -1)
  python3 tools/prof_summary.py "$T" --md "$OUT/kernel_summary_$W.md" > /dev/null
  echo "$W: rocprof done"
  timeout -k 10 400 python3 bench.py --workload $W $BENCH_ARGS > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err"
  echo "$W done: $(head -c 300 $OUT/bench_$W.json)"
done
echo "measure done"
