#!/bin/bash
# LDS-array / VALU busy fraction per kernel (GPU box): one PMC pass over a short single-stream bench run.
#   lds_busy  = SQ_LDS_IDX_ACTIVE / (CUs x GRBM_GUI_ACTIVE)   (LDS-array cycles per CU per elapsed cycle)
#   valu_busy = SQ_ACTIVE_INST_VALU / (4 SIMDs x CUs x GRBM_GUI_ACTIVE)
set -e
OUT=${1:-gpurun_out/ldsbusy}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d "$ROOT/$OUT/p" -o pmc -- python3 "$ROOT/bench.py" --batch 256 --streams 1 --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_EXTRA:-} > "$ROOT/$OUT/p.json" 2> "$ROOT/$OUT/p.err")
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if int(float(r["Grid_Size"])) < 20000: continue
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
CU = 256
for k, cs in sorted(acc.items()):
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    g = m.get("GRBM_GUI_ACTIVE", 0) or 1
    print(f"{k[:40]:40s} cyc {g:10.0f}  lds_busy {m.get('SQ_LDS_IDX_ACTIVE',0)/(CU*g):.3f}  conflict/active {m.get('SQ_LDS_BANK_CONFLICT',0)/max(m.get('SQ_LDS_IDX_ACTIVE',1),1):.3f}"
          f"  valu_busy {m.get('SQ_ACTIVE_INST_VALU',0)/(4*CU*g):.3f}  lds_inst_busy {m.get('SQ_ACTIVE_INST_LDS',0)/(CU*g):.3f}"
          f"  valu_insts {m.get('SQ_INSTS_VALU',0):.4g} lds_insts {m.get('SQ_INSTS_LDS',0):.4g} waves {m.get('SQ_WAVES',0):.4g} busy_cu {m.get('SQ_BUSY_CU_CYCLES',0)/(CU*g):.3f}")
PY
