set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -1 gpurun_out/tests.log
for i in 1 2 3; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names prev,late,new -- --workload stereo --steps 30; done > gpurun_out/rab.log 2>&1
cat gpurun_out/rab.log | python3 -c "
import sys, json
for l in sys.stdin:
    n, j = l.split(' ', 1); d = json.loads(j); print(n, d['value'], d['stages']['stereo'], d['stages']['describe'], d['parity']['mismatches'])"
