#!/bin/bash
# Latency / stall counters per kernel (GPU box): two PMC passes, each its own short bench run and time limit.
set -e
OUT=${1:-gpurun_out/stalls}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for grp in \
  "SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES" \
  "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVES SQ_INSTS_BRANCH"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/$OUT/p$i" -o pmc -- python3 "$ROOT/bench.py" --batch 128 --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/$OUT/p$i.json" 2> "$ROOT/$OUT/p$i.err")
  echo "pass $i done"
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if int(float(r["Grid_Size"])) < 20000: continue  # batch launches only
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    out = {c: f"{v:.4g}" for c, v in sorted(m.items())}
    lds_lat = m.get("SQ_INST_LEVEL_LDS", 0) / max(m.get("SQ_INSTS_LDS", 1), 1)
    vm_lat = m.get("SQ_INST_LEVEL_VMEM", 0) / max(m.get("SQ_INSTS_VMEM", 1), 1)
    print(k, f"LDS latency/instr {lds_lat:.1f} cyc, VMEM latency/instr {vm_lat:.1f} cyc")
    print("   ", out)
PY
