#!/bin/bash
# Round-5 closing suite (after the FAST stage-1 and pyramid SDWA changes) (GPU box, repo root): the whole GPU suite, smoke(), the headline bench line (default
# arguments: uninstrumented timed loop + instrumented pass + CPU baseline), single-frame latency, the FAST phase
# profile (fastprof variant), a 2-rank gloo rehearsal of config 3 on the one GPU, and a streams sweep
set -e
O=gpurun_out/final9
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
head -c 600 $O/bench_default.json; echo
timeout -k 10 300 python tools/latency.py --json $O/latency.json > $O/latency.log 2>&1 || { tail -20 $O/latency.log; exit 1; }
tail -5 $O/latency.log
timeout -k 10 200 python tools/fast_profile.py --run --batch 256 > $O/fast_profile.txt 2>&1 || true
head -12 $O/fast_profile.txt
ORBGPU_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 100 --warmup 3 > $O/rehearsal_2rank_gloo.json 2> $O/rehearsal.err || { tail -20 $O/rehearsal.err; exit 1; }
head -c 400 $O/rehearsal_2rank_gloo.json; echo
for S in 1 4; do timeout -k 10 300 python bench.py --streams $S --steps 300 --no-cpu-baseline > $O/bench_streams$S.json 2> $O/bench_streams$S.err || true; head -c 160 $O/bench_streams$S.json; echo; done
echo final-a done
