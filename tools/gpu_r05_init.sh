#!/bin/bash
# SearchForInitialization candidate grid limited to level-0 queries: the matcher tests with the working tree's library
# (in-tree liborbgpu.so), digests against the committed build (variant head), and the mono_init bench A/B.
set -e
OUT=gpurun_out/init
mkdir -p "$OUT"
export TMPDIR=/tmp
V=$PWD/orbslam2_with_quadrics_amd/variants
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_match.py tests/test_gpu_record.py tests/test_gpu_bench_shape.py tests/test_gpu_binding_matchers.py > "$OUT/tests.log" 2>&1
echo "tests: $(tail -1 $OUT/tests.log)"
ORBGPU_LIB=$V/liborbgpu_head.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_head.json" 2> "$OUT/probe_head.err"
ORBGPU_LIB=$V/liborbgpu_new.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_new.json" 2> "$OUT/probe_new.err"
cmp <(tail -1 "$OUT/probe_head.json") <(tail -1 "$OUT/probe_new.json")
echo "probe digests equal"
timeout -k 10 500 python3 tools/variant_bench.py --streams 2 --names head,new,head,new -- --steps 200 > "$OUT/ab_mono_init.txt" 2>&1
echo "all done"
