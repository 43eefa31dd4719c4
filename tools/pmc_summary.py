"""Aggregate rocprofv3 --pmc CSVs (tools/pmc_profile.sh) per bench STAGE for the B-frame launches and derive
per-launch metrics.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads 1/2 of the bytes of wide
coalesced streams on gfx950 -> doubled ("corrected"); WRITE_SIZE (KB) taken as is.

A stage's launch is every dispatch of its kernels for one batch: dispatches with a grid of at least 1/16 of the
kernel's largest grid belong to the B-frame batches (the 1-frame set-up extractions are 1/64 - 1/256 of it); a stage's
per-launch value = the sum over those dispatches / the number of batches (= B-frame FAST dispatches).

python tools/pmc_summary.py <pmc dir> [--json out.json] [--md out.md] [--batch B]
(--batch = frames per launch of the profiled bench run = batch / streams; bench.py rescales traffic if its
per-launch frame count differs)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(n):
    """Kernel name without arguments or template parameters (og_describe_kernel<0, false> -> og_describe_kernel)."""
    return n.split("(")[0].replace("void ", "").split("<")[0].strip()


# kernel -> bench stage (orbgpu_set_stage_timing's names, bench.py "stages_ms_per_launch")
STAGE = {"og_fast_quad_kernel": "fast", "og_octree_kernel": "octree",
         "og_octree_big_kernel": "octree", "og_describe_kernel": "describe", "og_grid_kernel": "grid",
         "og_resize_kernel": "pyramid", "og_resize2_kernel": "pyramid",
         "og_init_cand_kernel": "search_init", "og_init_resolve_kernel": "search_init",
         "og_stereo_rows_kernel": "stereo", "og_stereo_match16_kernel": "stereo",
         "og_stereo_filter_kernel": "stereo",
         "og_projb_count_kernel": "search_proj", "og_projb_scan_kernel": "search_proj",
         "og_projb_fill_kernel": "search_proj", "og_projb_resolve_kernel": "search_proj",
         "og_frustum_batch_kernel": "frustum"}
FAST = ("og_fast_quad_kernel",)


def main():
    d = sys.argv[1]
    # kernel -> list of (grid, {counter: value}) per dispatch
    disp = defaultdict(dict)
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (f, r.get("Dispatch_Id", r.get("Correlation_Id", "")))
            k = short(r["Kernel_Name"])
            e = disp[k].setdefault(key, {"grid": int(float(r["Grid_Size"])), "c": {}})
            e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # per kernel and counter: the sum over the batch dispatches, and the number of batches a counter was seen in
    # (each --pmc pass is its own run; a counter's batches are the FAST dispatches of that pass)
    per_kernel = {}
    for k, ds in disp.items():
        gmax = max(e["grid"] for e in ds.values())
        per_kernel[k] = [e for e in ds.values() if e["grid"] * 16 >= gmax]
    nb = defaultdict(int)  # counter -> B-frame FAST dispatches that report it
    for k in FAST:
        for e in per_kernel.get(k, []):
            for c in e["c"]:
                nb[c] += 1
    stages = defaultdict(lambda: defaultdict(float))
    for k, es in per_kernel.items():
        st = STAGE.get(k)
        if st is None:
            continue
        for e in es:
            for c, v in e["c"].items():
                stages[st][c] += v
    out = {}
    for st, cs in stages.items():
        m = {c: v / max(nb.get(c, 1), 1) for c, v in cs.items()}
        e = dict(m)
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            e["hbm_bytes_per_launch"] = int(2 * m.get("FETCH_SIZE", 0) * 1024 + m.get("WRITE_SIZE", 0) * 1024)
        if "SQ_INSTS_VALU" in m and m.get("SQ_WAVES"):
            e["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        if "SQ_INSTS_SALU" in m and m.get("SQ_WAVES"):
            e["salu_insts_per_wave"] = m["SQ_INSTS_SALU"] / m["SQ_WAVES"]
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if "SQ_ACTIVE_INST_VALU" in m and m.get("SQ_WAVE_CYCLES"):
            e["valu_active_frac_of_wave_cycles"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        out[st] = e
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 128
    js = {"source": d, "batch": batch, "note": "per-launch sums over each stage's kernels for one B-frame batch; "
                                "FETCH_SIZE doubled per the gfx950 correction (uncalibrated for non-16B accesses)",
          "kernels": out}
    if "--json" in sys.argv:
        json.dump(js, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    cols = ["waves", "VALU/wave", "SALU/wave", "LDS conflict", "VALU active", "wait", "HBM B/launch"]
    lines = ["| stage | " + " | ".join(cols) + " |", "|" + "---|" * (len(cols) + 1)]
    for k, e in sorted(out.items()):
        def g(x, fmt):
            return fmt.format(e[x]) if x in e else "-"
        lines.append(f"| {k} | {g('SQ_WAVES', '{:.0f}')} | {g('valu_insts_per_wave', '{:.0f}')} | "
                     f"{g('salu_insts_per_wave', '{:.0f}')} | {g('lds_bank_conflict_frac', '{:.3f}')} | "
                     f"{g('valu_active_frac_of_wave_cycles', '{:.3f}')} | {g('wait_frac', '{:.3f}')} | "
                     f"{g('hbm_bytes_per_launch', '{:.3e}')} |")
    md = "\n".join(lines)
    print(md)
    if "--md" in sys.argv:
        open(sys.argv[sys.argv.index("--md") + 1], "w").write(md + "\n")


if __name__ == "__main__":
    main()
