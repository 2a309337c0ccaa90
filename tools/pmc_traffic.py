#!/usr/bin/env python3
"""HBM traffic per bench step from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs).

The profiled command is `bench.py --config <leg> --steps S --warmup W --no-cpu-baseline
--no-extras`: every library dispatch of the run belongs to one of the S + W identical steps
(the generators and the copy-rate probe are torch kernels and are excluded by name), so
bytes per step = sum over the library's dispatches / (S + W).

Units and the gfx950 correction (MI355X_MICROARCH.md, HBM / rocprofv3): FETCH_SIZE and
WRITE_SIZE are in KB; FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read,
so reads are doubled; WRITE_SIZE is taken as reported.  Where the run contains k_part_hist,
whose reads are exactly 16 B x records (key + ts), the measured factor is reported beside the
guide's 2.0 as a check of the correction on this access pattern.

usage: pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <records>
                      <steps incl. warmup> <out json> <config key>
"""
import csv
import json
import re
import sys
from collections import defaultdict


def kname(raw):
    name = re.sub(r"\(.*", "", raw).replace("khip::", "").replace("void ", "")
    return re.sub(r"<.*", "", name).strip()


# library kernels that run outside the timed step of a leg (the join's table build)
OUTSIDE_STEP = ("k_upsert_claim", "k_upsert_finalize", "k_upsert_apply", "k_table_rehash", "k_count_live")


def library_kernel(name):
    # the library's kernels (torch's are at::native::...), minus the setup ones
    return name.startswith("k_") and name not in OUTSIDE_STEP


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = kname(r["Kernel_Name"])
        if library_kernel(name):
            per[name].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    n = int(sys.argv[3])
    steps = int(sys.argv[4])
    out_path, cfg = sys.argv[5], sys.argv[6]
    per_kernel = {}
    total = 0.0
    for k in sorted(set(fetch) | set(write)):
        rd = 2.0 * sum(fetch.get(k, [])) / steps
        wr = sum(write.get(k, [])) / steps
        per_kernel[k] = {"read_bytes_per_step": rd, "write_bytes_per_step": wr,
                         "dispatches_per_step": len(fetch.get(k, write.get(k, []))) / steps}
        total += rd + wr
    rec = {"records": n, "hbm_bytes_per_step": total, "hbm_bytes_per_record": total / n,
           "fetch_correction": 2.0, "per_kernel": per_kernel,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over the same bench "
                     "command; library kernels only; FETCH_SIZE x 2 (gfx950 wide-stream correction)"}
    hist = fetch.get("k_part_hist")
    if hist:
        rec["k_part_hist_fetch_factor_measured"] = (16.0 * n * len(hist) / steps) / sum(hist)
    try:
        prev = json.load(open(out_path))
    except (OSError, ValueError):
        prev = {}
    prev[cfg] = rec
    json.dump(prev, open(out_path, "w"), indent=1)
    print(json.dumps({cfg: {k: v for k, v in rec.items() if k != "per_kernel"}}, indent=1))


if __name__ == "__main__":
    main()
