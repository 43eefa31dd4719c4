#!/bin/bash
# Round-5 closing measurement (GPU box, repo root), after the last FAST change: PMC + kernel summaries + bench lines of
# all four workloads (tools/gpu_r05_measure.sh), then the serialised stereo pair's kernel summary.
set -e
bash tools/gpu_r05_measure.sh mono_init extract stereo tracking
timeout -k 10 400 bash tools/gpu_kstats.sh stereo_serial_pairs stereo --serial-pairs > /dev/null
cp gpurun_out/ks_stereo_serial_pairs/summary.md gpurun_out/meas/kernel_summary_stereo_serial_pairs.md
cp gpurun_out/ks_stereo_serial_pairs/kernel_stats.csv gpurun_out/meas/kernel_stats_stereo_serial_pairs_streams1.csv
echo "final-d done"
