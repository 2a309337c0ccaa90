#!/usr/bin/env python3
"""DESIGN.md's measurement table from bench JSON lines: one row per file (the last JSON line of
each), with records/s, ms/step, the byte basis of roofline.frac, frac, counter bytes per record
(roofline.traffic / records) and the CPU baseline at 1 / 4 / 16 threads.
usage: leg_table.py <label>=<file.jsonl>[@<traffic.json key>] ...  (@key: the counter bytes from
profiles/traffic.json instead of the line's own roofline.traffic, for lines run before the leg's
counters were measured)"""
import json
import sys


def rate(x):
    return "%.2e" % x if x else "—"


def main():
    print("| leg | records/s | ms/step | B/rec basis of frac | frac (wall) | counter B/rec | CPU 1 / 4 / 16 threads |")
    print("|---|---:|---:|---:|---:|---:|---|")
    for arg in sys.argv[1:]:
        label, path = arg.rsplit("=", 1)
        tkey = None
        if "@" in path:
            path, tkey = path.split("@", 1)
        d = [json.loads(l) for l in open(path) if l.startswith("{")][-1]
        r = d.get("roofline") or {}
        c = d.get("cpu_baseline") or {}
        cfg = d.get("config") or {}
        n = (cfg.get("records_per_gpu") or cfg.get("clicks_per_gpu") or cfg.get("rows_per_gpu") or
             cfg.get("records") or 0)
        tr = r.get("traffic")
        cb = "%.0f" % (tr / n) if tr and n else "—"
        if tkey:
            import os
            with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "traffic.json")) as f:
                cb = "%.0f" % json.load(f)[tkey]["hbm_bytes_per_record"]
        cpu = "—"
        if c:
            one = (c.get("single_thread") or {}).get("value")
            four = (c.get("ksql_default_threads") or {}).get("value")
            cpu = "%s / %s / %s" % (rate(one), rate(four), rate(c.get("value"))) if one else "%s (%d)" % (
                rate(c.get("value")), c.get("cores", 1))
        basis = r.get("algorithmic_bytes_per_record")
        print("| %s | %.2e | %.2f | %s | %.3f | %s | %s |" % (label, d["value"], d["ms_per_step"],
                                                           ("%.1f" % basis) if basis else "—", r.get("frac", 0.0), cb, cpu))


if __name__ == "__main__":
    main()
