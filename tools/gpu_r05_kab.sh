#!/bin/bash
# Kernel-level A/B (GPU box, repo root): probe digests of head and new, the extraction GPU tests on new, then the
# single-stream rocprof summary of config 3 for head and new (tools/gpu_kstats.sh with ORBGPU_LIB).
set -e
O=gpurun_out/kab
mkdir -p $O
export TMPDIR=/tmp
V=$PWD/orbslam2_with_quadrics_amd/variants
ORBGPU_LIB=$V/liborbgpu_head.so timeout -k 10 200 python3 tests/variant_probe.py > $O/probe_head.json 2> $O/probe_head.err
ORBGPU_LIB=$V/liborbgpu_new.so timeout -k 10 200 python3 tests/variant_probe.py > $O/probe_new.json 2> $O/probe_new.err
cmp <(tail -1 $O/probe_head.json) <(tail -1 $O/probe_new.json)
echo "probe digests equal"
ORBGPU_LIB=$V/liborbgpu_new.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_semantics.py tests/test_gpu_extract.py > $O/tests.log 2>&1
echo "tests: $(tail -1 $O/tests.log)"
for N in head new head new; do
  ORBGPU_LIB=$V/liborbgpu_$N.so timeout -k 10 400 bash tools/gpu_kstats.sh kab_$N mono_init > /dev/null
  echo "$N: $(grep 'og_resize_kernel\|og_resize2_kernel<false> \[6' gpurun_out/ks_kab_$N/summary.md | grep '| 512 |' | tr '\n' ' ')"
done
