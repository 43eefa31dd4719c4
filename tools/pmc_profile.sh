#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, never combined with tracing).
# Usage (on the GPU box, from the repo root): bash tools/pmc_profile.sh <outdir> [bench args...]
set -e
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
i=0
for grp in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" \
  "WRITE_SIZE" \
  "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$ROOT/$OUT/p$i" -o pmc -- python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/p$i.json" 2> "$ROOT/$OUT/p$i.err")
  echo "pass $i done: $grp"
done
