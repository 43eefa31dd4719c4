#!/bin/bash
# Per-(kernel, frames per launch) rocprof summary of a single-stream bench run (GPU box, repo root).
#   bash tools/gpu_kstats.sh <tag> <workload> [extra bench args...]
# -> gpurun_out/ks_<tag>/kernel_trace.csv, kernel_stats.csv and summary.md (tools/prof_summary.py: the 1-frame
#    set-up launches are listed on their own rows, never averaged into the B-frame launches)
set -e
TAG=$1; W=$2; shift 2
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/ks_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/raw" -o run \
    -- python3 "$ROOT/bench.py" --workload "$W" --streams 1 --steps 10 --warmup 2 --no-cpu-baseline "$@" \
    > "$OUT/bench.json" 2> "$OUT/err.log")
cp "$(find "$OUT/raw" -name '*kernel_trace.csv' | head -1)" "$OUT/kernel_trace.csv"
cp "$(find "$OUT/raw" -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats.csv"
rm -rf "$OUT/raw"
python3 "$ROOT/tools/prof_summary.py" "$OUT/kernel_trace.csv" --md "$OUT/summary.md" > /dev/null
cat "$OUT/summary.md"
