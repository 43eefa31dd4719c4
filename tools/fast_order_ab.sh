#!/bin/bash
# A/B of the FAST block-table order (ORBGPU_FAST_ORDER = XCD run length, orbgpu_capi.cpp build_plan), GPU box:
# bench FAST span per launch (config 3, 2 streams x 256 frames) and FAST HBM fetch / L2 hits from PMC passes.
set -e
OUT=gpurun_out/fast_order
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for R in ${@:-1 2 4 8}; do
  for rep in 1 2; do
    ORBGPU_FAST_ORDER=$R timeout -k 10 120 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline > "$OUT/bench_R${R}_$rep.json" 2> "$OUT/bench_R${R}_$rep.err"
  done
  i=0
  for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1)); tag=p$i
    (cd /tmp && ORBGPU_FAST_ORDER=$R timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/$OUT/pmc_R${R}/$tag" -o pmc -- python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$ROOT/$OUT/pmc_R${R}_$tag.err")
  done
  python3 tools/pmc_summary.py "$OUT/pmc_R${R}" --json "$OUT/pmc_R${R}.json" --batch 256 > /dev/null
  echo "R=$R done"
done
