#!/bin/bash
# Small-batch graph replay (GPU box, repo root): the whole GPU suite on the in-tree library (which replays graphs for
# batches <= 4), then the latency A/B against the previous build (tools/gpu_r05_latab.sh new).
set -e
O=gpurun_out/graph
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_r05_latab.sh new
