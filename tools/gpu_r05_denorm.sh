#!/bin/bash
# Round-5 session: VALU issue-rate microbenchmark, the denormal-f16 FAST encoding A/B (parity digest, then the bench
# alternating base/denorm at 1 and 2 streams), and the serialised stereo kernel profile.  Each GPU step has its own limit.
set -e
OUT=gpurun_out/dn
mkdir -p "$OUT"
export TMPDIR=/tmp
V=orbslam2_with_quadrics_amd/variants
timeout -k 10 120 ./tools/micro/valu_rate > "$OUT/valu_rate.txt" 2>&1
echo "valu_rate done"
ORBGPU_LIB=$V/liborbgpu_base.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_base.json" 2> "$OUT/probe_base.err"
ORBGPU_LIB=$V/liborbgpu_denorm.so timeout -k 10 200 python3 tests/variant_probe.py > "$OUT/probe_denorm.json" 2> "$OUT/probe_denorm.err"
cmp <(tail -1 "$OUT/probe_base.json") <(tail -1 "$OUT/probe_denorm.json")
echo "probe digests equal"
timeout -k 10 400 python3 tools/variant_bench.py --streams 1 --names base,denorm,base,denorm -- --steps 200 > "$OUT/ab_s1.txt" 2>&1
echo "ab s1 done"
timeout -k 10 400 python3 tools/variant_bench.py --streams 2 --names base,denorm,base,denorm -- --steps 200 > "$OUT/ab_s2.txt" 2>&1
echo "ab s2 done"
timeout -k 10 400 bash tools/gpu_kstats.sh stereo_serial stereo --serial-pairs > "$OUT/ks_stereo_serial.log" 2>&1
echo "all done"
