set -e
timeout -k 10 300 python tools/variant_parity.py --names rb22 > gpurun_out/bpar.log 2>&1 && tail -1 gpurun_out/bpar.log
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names bord0,rb8,rb22 -- --workload stereo --steps 30; done > gpurun_out/bab.log 2>&1
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names bord0,rb8,rb22 -- --steps 30; done >> gpurun_out/bab.log 2>&1
cat gpurun_out/bab.log | python3 -c "
import sys, json
for l in sys.stdin:
    n, j = l.split(' ', 1); d = json.loads(j); print(n, d['value'], d['stages']['fast'], d['stages']['describe'], d['parity']['mismatches'])"
