#!/bin/bash
# Round-5 measurement session (GPU box, repo root), for the given workloads (default all four):
#   1. PMC passes (tools/pmc_profile.sh) -> per-stage summary (tools/pmc_summary.py) -> profiles/pmc_latest[_<w>].json
#   2. single-stream rocprofv3 kernel trace -> per-(kernel, frames per launch) summary (tools/gpu_kstats.sh)
#   3. the default bench run of the workload (reads the fresh PMC file for roofline.traffic)
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
OUT=gpurun_out/meas
mkdir -p "$OUT"
export TMPDIR=/tmp
WORKLOADS=${@:-mono_init extract stereo tracking}
for W in $WORKLOADS; do
  P=$([ "$W" = mono_init ] && echo pmc_latest || echo pmc_latest_$W)
  timeout -k 10 400 bash tools/pmc_profile.sh "$OUT/pmc_$W" --workload $W --steps 3 --warmup 1 --no-cpu-baseline
  python3 tools/pmc_summary.py "$OUT/pmc_$W" --json "$OUT/$P.json" --md "$OUT/pmc_summary_$W.md" --batch 256
  cp "$OUT/$P.json" "profiles/$P.json"
  timeout -k 10 400 bash tools/gpu_kstats.sh "$W" "$W" > /dev/null
  cp gpurun_out/ks_$W/summary.md "$OUT/kernel_summary_$W.md"
  cp gpurun_out/ks_$W/kernel_stats.csv "$OUT/kernel_stats_${W}_streams1.csv"
  timeout -k 10 400 python3 bench.py --workload $W $BENCH_ARGS > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err"
  echo "$W done: $(head -c 200 $OUT/bench_$W.json)"
done
echo "measure done"
