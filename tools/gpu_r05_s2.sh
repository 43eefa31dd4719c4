#!/bin/bash
# Round 5 session 2: parity (matchers incl. the forced projection paths, every variant build and run-time switch,
# extraction), single-stream rocprof summaries (config 3; KITTI and 1080p frames on the single-context extract
# workload), per-level octree profiles of both shapes, then the whole GPU suite
set -e
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_variants.py tests/test_gpu_extract.py tests/test_gpu_bench_shape.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/t_s2.log 2>&1 || { tail -40 gpurun_out/r05/t_s2.log; exit 1; }
tail -2 gpurun_out/r05/t_s2.log
bash tools/gpu_kstats.sh mono mono_init > gpurun_out/r05/ks_mono.log 2>&1 && head -14 gpurun_out/r05/ks_mono.log
bash tools/gpu_kstats.sh kitti extract --rows 376 --cols 1241 --nfeatures 2000 > gpurun_out/r05/ks_kitti.log 2>&1 && head -12 gpurun_out/r05/ks_kitti.log
bash tools/gpu_kstats.sh hd extract --rows 1080 --cols 1920 --nfeatures 2000 > gpurun_out/r05/ks_hd.log 2>&1 && head -12 gpurun_out/r05/ks_hd.log
timeout -k 10 300 python tools/octree_profile.py --run --shape kitti --levels 0,1,2,3,4,5,6,7 --batch 64 > gpurun_out/r05/octprof_kitti.txt 2>&1 || true
timeout -k 10 300 python tools/octree_profile.py --run --levels 0,1,2,3,4,5,6,7 --batch 64 > gpurun_out/r05/octprof_hd.txt 2>&1 || true
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05/t_all.log 2>&1 || { tail -40 gpurun_out/r05/t_all.log; exit 1; }
tail -2 gpurun_out/r05/t_all.log
