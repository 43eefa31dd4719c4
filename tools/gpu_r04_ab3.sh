set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
for i in 1 2; do timeout -k 10 200 python tools/variant_bench.py --streams 2 --names dkold,dkupu,new -- --workload stereo --steps 30; done > gpurun_out/dkab2.log 2>&1
cat gpurun_out/dkab2.log
for i in 1 2; do timeout -k 10 200 python tools/variant_bench.py --streams 2 --names octold,new -- --steps 30; done > gpurun_out/octab.log 2>&1
cat gpurun_out/octab.log
