#!/bin/bash
# Per-kernel duration summary of a short bench run under rocprofv3 --kernel-trace --stats (GPU box).
# Usage: bash tools/kstats.sh <tag> [bench args...]
set -e
TAG=${1:-k}; shift || true
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/kstats_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
    -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/err.log")
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{float(r['AverageNs'])/1e3:10.1f} us  x{r['Calls']:>4}  {r['Name'][:90]}")
PY
python3 "$ROOT/tools/ktrace_groups.py" "$OUT" ${KGROUPS:-resize}
