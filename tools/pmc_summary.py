"""Median per-kernel SQ counters from a rocprofv3 counter_collection.csv: python tools/pmc_summary.py file.csv"""
import collections
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    by[r["Kernel_Name"].split("(")[0][-60:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in by.items():
    m = {c: statistics.median(v) for c, v in cs.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1) or 1
    line = " ".join(f"{c.replace('SQ_', '')}={v:.3g}" for c, v in sorted(m.items()))
    print(f"{k}\n   {line}")
    if "SQ_WAIT_ANY" in m:
        print(f"   wait_any/wave={m['SQ_WAIT_ANY'] / wc:.2f} wait_inst/wave={m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
              f"active/wave={m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} lds_conflict/lds_active="
              f"{m.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, m.get('SQ_LDS_IDX_ACTIVE', 1)):.2f} "
              f"mfma_busy/busy={m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(1, m.get('SQ_BUSY_CYCLES', 1)):.2f}")
