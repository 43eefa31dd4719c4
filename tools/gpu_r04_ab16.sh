set -e
for i in 1 2 3; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names prev,dk1,dk2 -- --workload stereo --steps 30; done > gpurun_out/rab.log 2>&1
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names prev,dk1,dk2 -- --steps 30; done >> gpurun_out/rab.log 2>&1
cat gpurun_out/rab.log | python3 -c "
import sys, json
for l in sys.stdin:
    n, j = l.split(' ', 1); d = json.loads(j); print(n, d['value'], d['stages']['fast'], d['stages']['describe'], d['parity']['mismatches'])"
