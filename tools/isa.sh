#!/bin/bash
# Device assembly of one source file (gfx950), with the build's flags: bash tools/isa.sh orb_extract.hip [-Dx=y ...]
# -> /tmp/isa_<file>.s ; prints each kernel's VGPR / SGPR / LDS / scratch from the assembly's metadata
set -e
SRC=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=/tmp/isa_${SRC%.*}.s
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
    -Wno-unused-result -Wno-comment -w "$@" -x hip --cuda-device-only -S "$ROOT/orbslam2_with_quadrics_amd/csrc/$SRC" -o "$OUT"
python3 - "$OUT" <<'PY'
import re, sys
s = open(sys.argv[1]).read()
for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n  - \.|\Z)", s, re.S):
    body = m.group(2)
    def g(k):
        r = re.search(r"\." + k + r":\s+(\d+)", body)
        return r.group(1) if r else "-"
    name = m.group(1)
    if "kernel" in name or name.startswith("_Z"):
        print(f"{name[:70]:70s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} lds {g('group_segment_fixed_size'):>6} "
              f"scratch {g('private_segment_fixed_size'):>4}")
PY
