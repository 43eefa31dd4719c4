#!/bin/bash
# Latency + throughput A/B of variant builds against head (GPU box, repo root).  Usage: bash tools/gpu_r05_latab.sh uc8,uc16
set -e
O=gpurun_out/latab
mkdir -p $O
export TMPDIR=/tmp
V=$PWD/orbslam2_with_quadrics_amd/variants
NAMES=${1:-new}
ORBGPU_LIB=$V/liborbgpu_head.so timeout -k 10 200 python3 tests/variant_probe.py > "$O/probe_head.json" 2> "$O/probe_head.err"
for N in ${NAMES//,/ }; do
  ORBGPU_LIB=$V/liborbgpu_$N.so timeout -k 10 200 python3 tests/variant_probe.py > "$O/probe_$N.json" 2> "$O/probe_$N.err"
  cmp <(tail -1 "$O/probe_head.json") <(tail -1 "$O/probe_$N.json")
  echo "probe digests equal: $N"
done
for i in 1 2; do
  for N in head ${NAMES//,/ }; do
    ORBGPU_LIB=$V/liborbgpu_$N.so timeout -k 10 300 python3 tools/latency.py --n 300 --json $O/lat_${N}_$i.json > $O/lat_${N}_$i.log 2>&1
    echo "latency $N $i: $(grep '^1920' $O/lat_${N}_$i.log | head -c 400)"
  done
done
timeout -k 10 600 python3 tools/variant_bench.py --streams 2 --names head,$NAMES,head,$NAMES -- --steps 200 --workload mono_init > "$O/ab_mono_init.txt" 2>&1
echo "all done"
