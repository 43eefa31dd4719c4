set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_projection.py tests/test_gpu_binding_matchers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pj_tests.log 2>&1 || { tail -20 gpurun_out/pj_tests.log; exit 1; }
tail -1 gpurun_out/pj_tests.log
for i in 1 2; do timeout -k 10 300 python tools/variant_bench.py --streams 2 --names pj0,pj1 -- --workload tracking --steps 30; done > gpurun_out/pjab.log 2>&1
cat gpurun_out/pjab.log | python3 -c "
import sys, json
for l in sys.stdin:
    n, j = l.split(' ', 1); d = json.loads(j); print(n, d['value'], d['stages']['search_proj'], d['parity']['mismatches'])"
