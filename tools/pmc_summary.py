"""Aggregate rocprofv3 --pmc CSVs (tools/pmc_profile.sh) per kernel for the B-frame launches and derive
per-launch metrics.  HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reads 1/2 of the bytes
of wide coalesced streams on gfx950 -> doubled ("corrected"); WRITE_SIZE (KB) taken as is.

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


STAGE = {"og_fast_blocks_kernel": "fast", "og_fast_persist_kernel": "fast", "og_fast_cells_kernel": "fast", "og_octree_kernel": "octree", "og_describe_kernel": "describe",
         "og_search_init_kernel": "search_init", "og_grid_kernel": "grid", "og_resize_kernel": "pyramid"}


def main():
    d = sys.argv[1]
    # kernel -> grid size -> counter -> [per-dispatch values]; the largest grid of a kernel is the
    # B-frame launch (the bench also extracts the 1-frame initial frame)
    raw = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            raw[k][int(float(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    vals = {}
    for k, by_grid in raw.items():
        if k.startswith("og_resize"):  # 7 levels per batch: keep all launches of the B-frame batch
            merged = defaultdict(list)
            for g, cs in by_grid.items():
                for c, v in cs.items():
                    merged[c].extend(v)
            vals[k] = merged
        else:
            vals[k] = by_grid[max(by_grid)]
    out = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        e = dict(m)
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            e["hbm_bytes_per_launch"] = int(2 * m.get("FETCH_SIZE", 0) * 1024 + m.get("WRITE_SIZE", 0) * 1024)
        if "SQ_INSTS_VALU" in m and "SQ_WAVES" in m and m["SQ_WAVES"]:
            e["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if "SQ_ACTIVE_INST_VALU" in m and m.get("SQ_WAVE_CYCLES"):
            e["valu_active_frac_of_wave_cycles"] = m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
            e["wait_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        out[STAGE.get(k, k)] = e
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 128
    js = {"source": d, "batch": batch, "note": "per-launch averages over the B-frame launches; FETCH_SIZE doubled per the "
                                "gfx950 correction (uncalibrated for non-16B accesses)", "kernels": out}
    if "--json" in sys.argv:
        json.dump(js, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    lines = ["| kernel | " + " | ".join(["waves", "VALU/wave", "LDS conflict", "VALU active", "wait", "HBM B/launch"]) + " |",
             "|---|---|---|---|---|---|---|"]
    for k, e in out.items():
        def g(x, fmt):
            return fmt.format(e[x]) if x in e else "-"
        lines.append(f"| {k} | {g('SQ_WAVES', '{:.0f}')} | {g('valu_insts_per_wave', '{:.0f}')} | "
                     f"{g('lds_bank_conflict_frac', '{:.3f}')} | {g('valu_active_frac_of_wave_cycles', '{:.3f}')} | "
                     f"{g('wait_frac', '{:.3f}')} | {g('hbm_bytes_per_launch', '{:.3e}')} |")
    md = "\n".join(lines)
    print(md)
    if "--md" in sys.argv:
        open(sys.argv[sys.argv.index("--md") + 1], "w").write(md + "\n")


if __name__ == "__main__":
    main()
