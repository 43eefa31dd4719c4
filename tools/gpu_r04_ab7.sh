set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_stereo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/st_tests.log 2>&1 || { tail -20 gpurun_out/st_tests.log; exit 1; }
tail -1 gpurun_out/st_tests.log
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names stu1,stu4,stu8 -- --workload stereo --steps 30; done > gpurun_out/stab.log 2>&1
cat gpurun_out/stab.log | python3 -c "
import sys, json
for l in sys.stdin:
    n, j = l.split(' ', 1); d = json.loads(j); print(n, d['value'], d['stages']['stereo'], d['stages']['describe'], d['parity']['mismatches'])"
