#!/usr/bin/env python3
"""Merge per-leg traffic summaries (profile_leg.sh → <dir>/<leg>/traffic.json) into
profiles/traffic.json, tagging each entry with the run it came from.
usage: merge_traffic.py <profiles/traffic.json> <run tag> <traffic.json>..."""
import json
import sys

out, tag, srcs = sys.argv[1], sys.argv[2], sys.argv[3:]
with open(out) as f:
    t = json.load(f)
for s in srcs:
    with open(s) as f:
        for k, v in json.load(f).items():
            v["source"] = "%s (%s)" % (tag, s.split("gpurun_out/")[-1])
            t[k] = v
            print(k, round(v["hbm_bytes_per_record"], 2))
with open(out, "w") as f:
    json.dump(t, f, indent=1, sort_keys=True)
    f.write("\n")
