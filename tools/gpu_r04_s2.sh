#!/bin/bash
set -e
OUT=gpurun_out/s2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python bench.py --workload tracking --steps 40 --no-cpu-baseline > $OUT/bench_tracking.json 2> $OUT/bench_tracking.err
python -c "import json;d=json.load(open('$OUT/bench_tracking.json'));print('tracking', d['value'], d['parity'], {k:round(x,3) for k,x in d['stages_busy_ms_per_step'].items()})"
timeout -k 10 400 bash tools/gpu_kstats.sh rows0 mono_init > /dev/null
ORBGPU_PYR_ROWS=1 timeout -k 10 400 bash tools/gpu_kstats.sh rows1 mono_init > /dev/null
timeout -k 10 400 bash tools/gpu_kstats.sh track tracking > /dev/null
for t in rows0 rows1 track; do echo "== $t"; head -16 gpurun_out/ks_$t/summary.md; done
timeout -k 10 200 python tools/fast_profile.py --run --batch 256 | tee $OUT/fast_profile.txt
