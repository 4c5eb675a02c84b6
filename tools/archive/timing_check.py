"""Cross-check of the bench's live HIP-event timing of the dominant kernel against the rocprofv3 kernel trace of the
same run (`tools/gpu_check.sh TAG prof`: bench.py --steps K --warmup W under rocprofv3 --kernel-trace).

In-step launches = the full-patch (2x96^3, 256-workgroup) conv32 ring forward launches (GN prologue, with or
without residual: the ones bench.py averages) of the K timed steps; standalone = the trailing 3 + 20 launches of bench.dominant_kernel_roofline
(each followed by its statistics finalize; the events there bracket both).
Usage: python tools/timing_check.py gpurun_out/TAG/kt gpurun_out/TAG/bench_kt.log STEPS OUT.json"""
import glob
import json
import sqlite3
import statistics
import sys

kt, log, steps, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
dbs = glob.glob(f"{kt}/**/*.db", recursive=True)
if dbs:
    rows = list(sqlite3.connect(dbs[0]).execute("select name, start, end, grid_x from kernels order by start"))
else:  # --output-format csv
    import csv
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"]))
                   for r in csv.DictReader(open(glob.glob(f"{kt}/**/*kernel_trace.csv", recursive=True)[0]))),
                  key=lambda r: r[1])
fwd = [i for i, r in enumerate(rows) if "conv32_ring_kernel<false, true" in r[0] and r[3] >= 256 * 512]
line = json.loads([l for l in open(log) if l.startswith("{")][-1])
roof = line["roofline"]
nev = int(roof["timing"].split(",")[1].split()[0])  # "HIP events, N launches, ..." (full-patch launches only)
alone, in_step = fwd[-23:], fwd[:-23][-nev:]
dur = lambda i: (rows[i][2] - rows[i][1]) / 1e3  # noqa: E731
t_alone = [(rows[i + 1][2] - rows[i][1]) / 1e3 for i in alone[3:]]  # conv + finalize, as the events bracket them
res = {
    "source": {"trace": kt, "bench_line": log},
    "in_step_launches": len(in_step),
    "in_step_events_us": round(roof["avg_launch_ms"] * 1e3, 1),
    "in_step_trace_us": round(statistics.mean(dur(i) for i in in_step), 1),
    "standalone_events_us": round(roof["standalone_launch_ms"] * 1e3, 1),
    "standalone_trace_us": round(statistics.mean(t_alone), 1),
    "standalone_trace_kernel_only_us": round(statistics.mean(dur(i) for i in alone[3:]), 1),
    "bench_ms_per_step_under_rocprof": line["ms_per_step"],
}
res["in_step_trace_over_events"] = round(res["in_step_trace_us"] / res["in_step_events_us"], 3)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
