#!/bin/bash
# PMC A/B of experiment libraries (orbslam2_with_quadrics_amd/variants/liborbgpu_<name>.so): the two SQ counter
# groups of tools/pmc_profile.sh per library, one rocprofv3 --pmc pass each (GPU box, repo root).
# Usage: bash tools/pmc_ab.sh <outdir> name1 name2 ...
set -e
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
for name in "$@"; do
  i=0; mkdir -p "$OUT/$name"
  for grp in \
    "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
    "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    (cd /tmp && ORBGPU_LIB="$ROOT/orbslam2_with_quadrics_amd/variants/liborbgpu_$name.so" timeout -k 10 120 \
      rocprofv3 --pmc $grp --output-format csv -d "$ROOT/$OUT/$name/p$i" -o pmc -- python3 "$ROOT/bench.py" \
      --steps 3 --warmup 1 --no-cpu-baseline > "$ROOT/$OUT/$name/p$i.json" 2> "$ROOT/$OUT/$name/p$i.err")
  done
  python3 tools/pmc_summary.py "$OUT/$name" --json "$OUT/$name.json" --batch ${PMC_BATCH:-512} > /dev/null
  python3 -c "
import json,sys; k=json.load(open('$OUT/$name.json'))['kernels']['fast']
print('$name', ' '.join('%s=%.4g' % (c, k[c]) for c in ('SQ_WAVES','SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_WAVE_CYCLES','SQ_WAIT_ANY','SQ_WAIT_INST_ANY','SQ_ACTIVE_INST_ANY','SQ_LDS_BANK_CONFLICT','SQ_LDS_IDX_ACTIVE','GRBM_GUI_ACTIVE') if c in k))
"
done
