#!/bin/bash
# One measurement session on the GPU box (run from the repo root through gpurun):
#   1. PMC passes (tools/pmc_profile.sh) -> per-kernel HBM bytes -> profiles/pmc_latest.json (box copy)
#   2. bench.py default run (N=1) -> gpurun_out/meas/bench.json (picks up the PMC traffic)
#   3. rocprofv3 --kernel-trace --stats of a shorter bench run -> kernel stats CSV
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
OUT=gpurun_out/meas
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 600 bash tools/pmc_profile.sh "$OUT/pmc"
python3 tools/pmc_summary.py "$OUT/pmc" --json "$OUT/pmc_latest.json" --md "$OUT/pmc_summary.md" --batch 256
cp "$OUT/pmc_latest.json" profiles/pmc_latest.json
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$ROOT/$OUT/bench_under_rocprof.json" \
    2> "$ROOT/$OUT/rocprof.err")
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
echo "measure done"
