"""Per-(kernel, grid) average durations from a rocprofv3 --kernel-trace CSV (test infrastructure).
Usage: python tools/ktrace_groups.py <dir with *kernel_trace.csv> [name substring ...]"""
import collections
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
keys = sys.argv[2:]
g = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(")[0]
    if keys and not any(k in n for k in keys):
        continue
    wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
    grid = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]) // int(r["Workgroup_Size_Y"]),
            int(r["Grid_Size_Z"]) // int(r["Workgroup_Size_Z"]))
    g[(n, wg, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, wg, grid), v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / len(v):10.1f} us  x{len(v):>4}  wg {wg:>4}  grid {grid}  {n[:60]}")
