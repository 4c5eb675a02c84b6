"""Print rows of rocprofv3 kernel_stats CSVs matching a regex: tools/kstats.py REGEX file.csv [file2.csv ...]
(name shortened to its template head; calls, total ms, average us)."""
import csv
import re
import sys

rx = re.compile(sys.argv[1])
for path in sys.argv[2:]:
    print(f"== {path}")
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Name"]
            if rx.search(name):
                short = name.split("(")[0].replace("void ", "").replace("u3d::", "")
                print(f"  {short[:70]:70s} calls {int(row['Calls']):5d}  total {int(row['TotalDurationNs']) / 1e6:8.3f} ms"
                      f"  avg {float(row['AverageNs']) / 1e3:8.1f} us")
