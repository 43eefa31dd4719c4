#!/bin/bash
# HBM fetch A/B of experiment libraries (orbslam2_with_quadrics_amd/variants/liborbgpu_<name>.so): one
# rocprofv3 --pmc FETCH_SIZE pass per library (WRITE_SIZE needs a run of its own: 3 + 2 TCC counters > 4) over a short default bench run, summarised per stage
# (tools/pmc_summary.py; FETCH_SIZE doubled per MI355X_MICROARCH.md).  GPU box, repo root.
# Usage: bash tools/fetch_ab.sh <outdir> name1 name2 ...
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for name in "$@"; do
  mkdir -p "$OUT/$name"
  (cd /tmp && ORBGPU_LIB="$ROOT/orbslam2_with_quadrics_amd/variants/liborbgpu_$name.so" timeout -k 10 120 \
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOT/$OUT/$name/p1" -o pmc -- python3 "$ROOT/bench.py" \
    --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/$OUT/$name/p1.json" 2> "$ROOT/$OUT/$name/p1.err")
  python3 tools/pmc_summary.py "$OUT/$name" --json "$OUT/$name.json" --batch ${PMC_BATCH:-512} > /dev/null
  python3 -c "
import json; k=json.load(open('$OUT/$name.json'))['kernels']
print('$name', {s: round(k[s]['FETCH_SIZE'] * 2 * 1024 / 1e9, 3) for s in ('fast', 'pyramid', 'describe', 'octree') if s in k}, 'GB fetched per launch (FETCH_SIZE KB x 2)')
"
done
