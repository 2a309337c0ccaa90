#!/usr/bin/env python3
"""Print one bench step's kernel timeline (start, duration, gap before) from a rocprofv3
kernel_trace.csv: from the second-to-last occurrence of the first kernel named in argv[2]."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "k_part_reset"
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
i0 = idx[-2]
t0 = prev = int(rows[i0]["Start_Timestamp"])
end = idx[-1]
for r in rows[i0:end + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f %8.1f gap %6.1f %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3, r["Kernel_Name"][:70]))
    prev = e
