#!/bin/bash
# A/B of several working-tree variants against head: probe digests of each, the extraction GPU tests on "new", and
# tools/variant_bench.py on mono_init.  Usage: bash tools/gpu_r05_ab3.sh new,new4
set -e
OUT=gpurun_out/ab
mkdir -p "$OUT"
export TMPDIR=/tmp
V=$PWD/orbslam2_with_quadrics_amd/variants
NAMES=${1:-new}
ORBGPU_LIB=$V/liborbgpu_head.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_head.json" 2> "$OUT/probe_head.err"
for N in ${NAMES//,/ }; do
  ORBGPU_LIB=$V/liborbgpu_$N.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_$N.json" 2> "$OUT/probe_$N.err"
  cmp <(tail -1 "$OUT/probe_head.json") <(tail -1 "$OUT/probe_$N.json")
  echo "probe digests equal: $N"
done
ORBGPU_LIB=$V/liborbgpu_new.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_semantics.py tests/test_gpu_extract.py > "$OUT/tests.log" 2>&1
echo "tests: $(tail -1 $OUT/tests.log)"
timeout -k 10 700 python3 tools/variant_bench.py --streams 2 --names head,$NAMES,head,$NAMES -- --steps 200 --workload mono_init > "$OUT/ab_mono_init.txt" 2>&1
echo "all done"
