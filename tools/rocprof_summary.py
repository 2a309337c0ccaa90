#!/usr/bin/env python3
"""Summarize rocprofv3 CSV output (kernel stats / kernel trace / counter collection).

usage: rocprof_summary.py stats <run_kernel_stats.csv>
       rocprof_summary.py pmc <run_counter_collection.csv> [kernel-regex]
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("khip::", "")


def stats(path):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("| kernel | calls | avg us | total ms | % |")
    print("|---|---:|---:|---:|---:|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        print("| %s | %s | %.1f | %.3f | %.1f |" % (short(r["Name"])[:70], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                    float(r["TotalDurationNs"]) / 1e6,
                                                    100 * float(r["TotalDurationNs"]) / tot))


def pmc(path, rx=None):
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(lambda: defaultdict(list))
    for r in rows:
        k = short(r.get("Kernel_Name", r.get("Kernel-Name", "")))
        if rx and not re.search(rx, k):
            continue
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in agg.items():
        for c, v in cs.items():
            print("%s %s dispatches=%d mean_per_dispatch=%.6g" % (k, c, len(v), sum(v) / len(v)))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2])
    else:
        pmc(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
