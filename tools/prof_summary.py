"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, batch size) -- average launch duration,
VGPR/SGPR/LDS, and the launch count -- so the bench's HIP-event stage times can be checked against the
profiler for the B-frame launches (the bench also launches 1-frame extractions of the initial frame).

python tools/prof_summary.py <kernel_trace.csv> [--md out.md]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    path = sys.argv[1]
    md = sys.argv[sys.argv.index("--md") + 1] if "--md" in sys.argv else None
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: [0, 0.0, None])
    for r in rows:
        if r["Kind"] != "KERNEL_DISPATCH":
            continue
        k = short(r["Kernel_Name"])
        gx, gy, gz = int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"])
        wx, wy, wz = int(r["Workgroup_Size_X"]), int(r["Workgroup_Size_Y"]), int(r["Workgroup_Size_Z"])
        # frames per launch: z for the pyramid kernel, x/8 for the octree, x for the matchers, x * z for FAST (frame
        # chunks of up to 64 on x, chunks on z: B rounded up to a chunk multiple), y for the others
        if k.startswith("og_fast_quad"):
            batch = gx // max(wx, 1) * gz
        elif k.startswith("og_resize"):
            batch = gz // max(wz, 1)
        elif k.startswith("og_octree"):  # level-major 1-D grid: 8 levels x B frames (the single-frame fork splits
            batch = max(1, round(gx // max(wx, 1) / 8))  # level 0 from levels 1-7: 1 and 7 workgroups, one frame)
        elif k.startswith(("og_search_init", "og_grid", "og_init_resolve", "og_projb_resolve", "og_stereo_rows",
                            "og_stereo_filter")):
            batch = gx // max(wx, 1)
        else:
            batch = gy // max(wy, 1)
        # the pyramid's fused launches ((1,2), (3,4), (5,6)) differ in their tile grid: one row each
        key = (k + (f" [{gx // max(wx, 1)}x{gy // max(wy, 1)}]" if k.startswith("og_resize") else ""), batch)
        a = agg[key]
        a[0] += 1
        a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        a[2] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size_X"])
    lines = ["| kernel | frames per launch | launches | avg ms | VGPR | SGPR | LDS B | WG |",
             "|---|---|---|---|---|---|---|---|"]
    for (k, b), (n, tot, res) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"| {k} | {b} | {n} | {tot / n:.4f} | {res[0]} | {res[1]} | {res[2]} | {res[3]} |")
    out = "\n".join(lines)
    print(out)
    if md:
        open(md, "w").write(out + "\n")


if __name__ == "__main__":
    main()
