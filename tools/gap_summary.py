"""Per-step GPU wall vs busy time from a rocprofv3 kernel trace (steps delimited by the SGD kernel launches):
idle = wall - busy (union of kernel intervals), plus the largest idle gaps and the kernels that follow them.
Usage: python tools/gap_summary.py run_kernel_trace.csv [skip_steps]"""
import csv
import sys


def main(path, skip=3):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    sgd_idx = [i for i, e in enumerate(ev) if "sgd_kernel" in e[2]]
    # a step ends at the last SGD launch of a run of consecutive SGD kernels
    ends = [i for k, i in enumerate(sgd_idx) if k + 1 == len(sgd_idx) or sgd_idx[k + 1] != i + 1]
    steps = list(zip(ends[skip:-1], ends[skip + 1:]))
    tot_wall = tot_busy = 0
    gaps = []
    for a, b in steps:
        seg = ev[a + 1:b + 1]
        t0, t1 = seg[0][0], max(e[1] for e in seg)
        busy, cur_s, cur_e = 0, seg[0][0], seg[0][1]
        prev_end = seg[0][1]
        for s, e, n in seg[1:]:
            if s > prev_end:
                gaps.append((s - prev_end, n[:70]))
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev_end = max(prev_end, e)
        busy += cur_e - cur_s
        tot_wall += t1 - t0
        tot_busy += busy
    n = len(steps)
    print(f"steps {n}: wall {tot_wall / n / 1e6:.3f} ms/step, busy {tot_busy / n / 1e6:.3f}, idle {(tot_wall - tot_busy) / n / 1e6:.3f}")
    gaps.sort(reverse=True)
    tot = sum(g for g, _ in gaps)
    print(f"gaps: {len(gaps) / n:.0f} per step, {tot / n / 1e3:.0f} us/step; >20us: "
          f"{sum(g for g, _ in gaps if g > 20000) / n / 1e3:.0f} us/step")
    for g, name in gaps[:12]:
        print(f"  {g / 1e3:8.1f} us before {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 3)
