"""Summarise a rocprofv3 --kernel-trace csv: per-kernel totals per step and the top (kernel, grid) groups."""
import collections
import csv
import sys

d = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
import glob
import os
import sqlite3


def load(d):
    """Kernel dispatch rows from a rocprofv3 output dir: csv (run_kernel_trace.csv) or the rocpd SQLite db."""
    if os.path.exists(f"{d}/run_kernel_trace.csv"):
        return list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    out = []
    for db in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        for name, st, en, gx, gy, gz, wx in c.execute(
                "select name, start, end, grid_x, grid_y, grid_z, workgroup_x from kernels"):
            out.append({"Kernel_Name": name, "Start_Timestamp": st, "End_Timestamp": en, "Grid_Size_X": gx,
                        "Grid_Size_Y": gy, "Grid_Size_Z": gz, "Workgroup_Size_X": wx})
    return out


rows = load(d)
if len(sys.argv) > 4 and sys.argv[4].startswith("steady"):  # only the last `steps` complete (timed) steps
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import trace_steps
    rows, walls, steps = trace_steps.steady(rows, steps)
    print(f"steady state: the last {steps} complete steps, wall per step {sum(walls) / len(walls) / 1e3:.3f} ms "
          f"(min {min(walls) / 1e3:.3f}, max {max(walls) / 1e3:.3f})")
tot = collections.defaultdict(float)
grp = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot[n] += dt
    k = (n[-70:], int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"], r["Grid_Size_Z"])
    grp[k][0] += 1
    grp[k][1] += dt
s = sum(tot.values())
print(f"GPU busy per step: {s / steps / 1e3:.3f} ms")
for n, v in sorted(tot.items(), key=lambda kv: -kv[1])[:18]:
    print(f"{v / steps / 1e3:8.3f} ms/step {100 * v / s:5.1f}%  {n[-90:]}")
print("--- top (kernel, grid) groups")
for k, v in sorted(grp.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 20]:
    print(f"{v[1] / steps / 1e3:7.3f} ms/step n/step={v[0] // steps:3d} avg={v[1] / v[0]:8.1f}us {k}")
