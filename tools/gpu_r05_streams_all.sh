#!/bin/bash
# --streams 1 vs 2 for every workload (GPU box, repo root), alternated twice, no CPU baseline.
set -e
O=gpurun_out/streams_all
mkdir -p $O
for W in mono_init extract stereo tracking; do
  for i in 1 2; do
    for S in 2 1; do
      timeout -k 10 300 python bench.py --workload $W --streams $S --no-cpu-baseline > $O/${W}_s${S}_$i.json 2> $O/${W}_s${S}_$i.err
      echo "$W streams $S run $i: $(python -c "import json; j=json.loads(open('$O/${W}_s${S}_$i.json').read().strip().splitlines()[-1]); print(j['value'], j['ms_per_step'], j['parity']['mismatches'])")"
    done
  done
done
