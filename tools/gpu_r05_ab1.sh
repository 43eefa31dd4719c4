#!/bin/bash
# Round 5 A/B session: wave-per-cell FAST (quad -> cell), pyramid A-pass row reuse (rz0 -> cell), describe with two
# keypoints per wave (dk1 -> dk2 = the default build); each variant's bench line carries its own parity check
# (hashes of every timed frame), then the extraction/matcher parity tests, a single-stream rocprof summary and the
# whole GPU suite on the default build
set -e
mkdir -p gpurun_out/r05
for i in 1 2; do timeout -k 10 400 python tools/variant_bench.py --streams 2 --names quad,cell,rz0,dk1,dk2,kb2w4,dma2w4 -- --steps 100; done > gpurun_out/r05/ab_mono.log 2>&1 || { tail -20 gpurun_out/r05/ab_mono.log; exit 1; }
cat gpurun_out/r05/ab_mono.log
timeout -k 10 400 python tools/variant_bench.py --streams 2 --names quad,cell,dk1,dk2 -- --workload stereo --steps 100 > gpurun_out/r05/ab_stereo.log 2>&1 || { tail -20 gpurun_out/r05/ab_stereo.log; exit 1; }
cat gpurun_out/r05/ab_stereo.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_extract.py tests/test_gpu_bench_shape.py tests/test_gpu_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/t_ext.log 2>&1 || { tail -40 gpurun_out/r05/t_ext.log; exit 1; }
tail -2 gpurun_out/r05/t_ext.log
bash tools/gpu_kstats.sh dflt mono_init > gpurun_out/r05/ks_dflt.log 2>&1 && head -16 gpurun_out/r05/ks_dflt.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r05/t_all.log 2>&1 || { tail -40 gpurun_out/r05/t_all.log; exit 1; }
tail -2 gpurun_out/r05/t_all.log
# clean single-context per-kernel times of KITTI and 1080p frames (the stereo workload runs its L and R contexts on two
# streams, so its rocprof durations overlap), and the octree's per-round profile at every level of both
bash tools/gpu_kstats.sh kitti extract --rows 376 --cols 1241 --nfeatures 2000 > gpurun_out/r05/ks_kitti.log 2>&1 && head -14 gpurun_out/r05/ks_kitti.log
bash tools/gpu_kstats.sh hd extract --rows 1080 --cols 1920 --nfeatures 2000 > gpurun_out/r05/ks_hd.log 2>&1 && head -14 gpurun_out/r05/ks_hd.log
timeout -k 10 300 python tools/octree_profile.py --run --shape kitti --levels 0,1,2,3,4,5,6,7 --batch 64 > gpurun_out/r05/octprof_kitti.txt 2>&1 || true
timeout -k 10 300 python tools/octree_profile.py --run --levels 0,1,2,3,4,5,6,7 --batch 64 > gpurun_out/r05/octprof_hd.txt 2>&1 || true
