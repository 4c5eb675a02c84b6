"""Median per-kernel SQ counters from a rocprofv3 counter_collection.csv: python tools/pmc_summary.py file.csv

mfma_busy is SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over every SIMD of the chip: = 16 x N for
v_mfma_f32_16x16x32_bf16) divided by SIMD-cycles of the launch: 1024 SIMDs (256 CUs x 4) x the kernel's cycles, the
latter GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs; MI355X_MICROARCH.md, DVFS and counter-unit
rows). That fraction is comparable with the bench's roofline frac (it prices the launch at the clock it ran at)."""
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
              + (f"mfma_busy/(1024 SIMDs x GRBM_GUI_ACTIVE/8)="
                 f"{m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) * 8 / (1024 * m['GRBM_GUI_ACTIVE']):.3f} "
                 f"(kernel cycles {m['GRBM_GUI_ACTIVE'] / 8:.4g})" if m.get("GRBM_GUI_ACTIVE") else
                 "mfma_busy: GRBM_GUI_ACTIVE not collected"))
