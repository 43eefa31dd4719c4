set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 400 bash tools/pmc_profile.sh gpurun_out/pmc_oct --workload mono_init --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_oct.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_oct --md gpurun_out/pmc_oct.md --batch 256 > /dev/null && grep octree gpurun_out/pmc_oct.md
timeout -k 10 400 bash tools/pmc_profile.sh gpurun_out/pmc_oct5 --workload tracking --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_oct5.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_oct5 --md gpurun_out/pmc_oct5.md --batch 256 > /dev/null && grep octree gpurun_out/pmc_oct5.md
for i in 1 2; do timeout -k 10 200 python tools/variant_bench.py --streams 2 --names octold,new -- --steps 30; done > gpurun_out/octab.log 2>&1
for i in 1 2; do timeout -k 10 200 python tools/variant_bench.py --streams 2 --names octold,new -- --workload tracking --steps 30; done >> gpurun_out/octab.log 2>&1
cat gpurun_out/octab.log | python3 -c "
import sys, json
for l in sys.stdin:
    n, j = l.split(' ', 1); d = json.loads(j); print(n, d['value'], d['stages']['octree'], d['parity']['mismatches'])"
timeout -k 10 60 ./tools/issue_probe > gpurun_out/issue_probe.jsonl && cat gpurun_out/issue_probe.jsonl
