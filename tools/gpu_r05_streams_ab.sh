#!/bin/bash
# Streams A/B of the headline configuration (GPU box, repo root): bench.py at --streams 1 and 2, alternated three
# times, 500 timed steps each, no CPU baseline.
set -e
O=gpurun_out/streams_ab
mkdir -p $O
for i in 1 2 3; do
  for S in 2 1; do
    timeout -k 10 300 python bench.py --streams $S --steps 500 --no-cpu-baseline > $O/s${S}_$i.json 2> $O/s${S}_$i.err
    echo "streams $S run $i: $(python -c "import json,sys; j=json.loads(open('$O/s${S}_$i.json').read().strip().splitlines()[-1]); print(j['value'], j['ms_per_step'], j['parity']['mismatches'])")"
  done
done
