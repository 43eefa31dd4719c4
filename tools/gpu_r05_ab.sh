#!/bin/bash
# A/B of the working tree (variant "new") against the committed kernels (variant "head"): tests/variant_probe.py
# digests, the extraction / semantics GPU tests, and tools/variant_bench.py on the given workloads (default mono_init
# tracking).  Each GPU step has its own limit; the script stops at the first failure.
set -e
OUT=gpurun_out/ab
mkdir -p "$OUT"
export TMPDIR=/tmp
V=$PWD/orbslam2_with_quadrics_amd/variants
WORKLOADS=${@:-mono_init tracking}
ORBGPU_LIB=$V/liborbgpu_head.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_head.json" 2> "$OUT/probe_head.err"
ORBGPU_LIB=$V/liborbgpu_new.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_new.json" 2> "$OUT/probe_new.err"
cmp <(tail -1 "$OUT/probe_head.json") <(tail -1 "$OUT/probe_new.json")
echo "probe digests equal"
ORBGPU_LIB=$V/liborbgpu_new.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_semantics.py tests/test_gpu_extract.py > "$OUT/tests.log" 2>&1
echo "tests: $(tail -1 $OUT/tests.log)"
for W in $WORKLOADS; do
  timeout -k 10 500 python3 tools/variant_bench.py --streams 2 --names head,new,head,new -- --steps 200 --workload $W > "$OUT/ab_$W.txt" 2>&1
  echo "ab $W done"
done
echo "all done"
