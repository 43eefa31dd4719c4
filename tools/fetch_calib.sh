#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over tools/fetch_calib (GPU box, repo root; build it here first:
# hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib).  One counter per pass.
set -e
OUT=gpurun_out/fetch_calib
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 60 ./tools/fetch_calib > $OUT/meta.json
for c in FETCH_SIZE TCC_EA0_RDREQ_sum; do
  (cd /tmp && timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$ROOT/$OUT/$c" -o pmc -- "$ROOT/tools/fetch_calib" > /dev/null)
done
python3 - <<'PY'
import csv, glob, json
meta = json.load(open("gpurun_out/fetch_calib/meta.json"))
res = {}
for c in ("FETCH_SIZE", "TCC_EA0_RDREQ_sum"):
    f = glob.glob(f"gpurun_out/fetch_calib/{c}/**/*counter_collection.csv", recursive=True)[0]
    agg = {}
    for r in csv.DictReader(open(f)):  # one dispatch may span several rows (summed, as tools/pmc_summary.py does)
        d = int(r.get("Dispatch_Id", r.get("Correlation_Id")))
        agg[d] = agg.get(d, 0.0) + float(r["Counter_Value"])
    res[c] = [agg[d] for d in sorted(agg)]
# dispatch order: the rocclr fill, stream4, stream8, stream16 (x2 reps), then tile_halo, tile_nohalo (x2 reps); the
# second rep of each kernel is the measured one
seq = ["fill", "stream4", "stream8", "stream16", "stream4", "stream8", "stream16", "tile_halo", "tile_nohalo",
       "tile_halo", "tile_nohalo"]
last = {}
for i, name in enumerate(seq):
    if name != "fill":
        last[name] = {c: res[c][i] for c in res}
req = {"stream4": meta["stream_bytes"], "stream8": meta["stream_bytes"], "stream16": meta["stream_bytes"],
       "tile_halo": meta["tile_halo_bytes_requested"], "tile_nohalo": meta["tile_nohalo_bytes_requested"]}
out = {}
for k, v in last.items():
    fb = v["FETCH_SIZE"] * 1024
    out[k] = {"requested_bytes": req[k], "FETCH_SIZE_bytes": fb, "fetch_x2_over_requested": 2 * fb / req[k],
              "rdreq_x128_bytes": v["TCC_EA0_RDREQ_sum"] * 128,
              "unique_bytes": meta["tile_unique_bytes"] if k.startswith("tile") else req[k]}
    out[k]["fetch_x2_over_unique"] = 2 * fb / out[k]["unique_bytes"]
json.dump(out, open("gpurun_out/fetch_calib/calib.json", "w"), indent=1)
for k, v in out.items():
    print(k, {a: round(b, 3) if isinstance(b, float) else b for a, b in v.items()})
PY
