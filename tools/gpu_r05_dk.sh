#!/bin/bash
# Round-5 session: describe with magic-number rounding and alignbyte tap weights (variant dkmagic = the working tree)
# against the committed kernel (variant base): digests, the semantics / describe GPU tests, bench A/B and single-stream
# kernel times.  Each GPU step has its own limit; the script stops at the first failure.
set -e
OUT=gpurun_out/dk
mkdir -p "$OUT"
export TMPDIR=/tmp
V=orbslam2_with_quadrics_amd/variants
ORBGPU_LIB=$V/liborbgpu_base.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_base.json" 2> "$OUT/probe_base.err"
timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_new.json" 2> "$OUT/probe_new.err"
cmp <(tail -1 "$OUT/probe_base.json") <(tail -1 "$OUT/probe_new.json")
echo "probe digests equal"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_semantics.py tests/test_gpu_extract.py > "$OUT/tests.log" 2>&1
echo "tests: $(tail -1 $OUT/tests.log)"
timeout -k 10 500 python3 tools/variant_bench.py --streams 2 --names base,dkmagic,base,dkmagic -- --steps 200 > "$OUT/ab_mono.txt" 2>&1
echo "ab mono done"
timeout -k 10 500 python3 tools/variant_bench.py --streams 2 --names base,dkmagic,base,dkmagic -- --steps 200 --workload tracking > "$OUT/ab_tracking.txt" 2>&1
echo "ab tracking done"
for n in base dkmagic; do
  ORBGPU_LIB=$PWD/$V/liborbgpu_$n.so timeout -k 10 400 bash tools/gpu_kstats.sh dk_$n mono_init > /dev/null
  cp gpurun_out/ks_dk_$n/summary.md "$OUT/ks_$n.md"
done
echo "all done"
