#!/usr/bin/env python3
"""HBM traffic per push from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs).

FETCH_SIZE/WRITE_SIZE are in KB.  On gfx950 FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads (MI355X_MICROARCH.md, HBM); we calibrate on k_part_hist, whose
reads are exactly 16 B x records (key + ts), and apply that factor to every kernel's reads.
WRITE_SIZE is taken as reported.

usage: pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <records>
                      <out json> [config]
"""
import csv
import json
import re
import sys
from collections import defaultdict

PUSH = ["k_part_hist", "k_part_colsum", "k_part_colbase", "k_part_colprefix", "k_scan_blocks", "k_scan_excl",
        "k_part_scatter", "k_part_refine", "k_part_wrange", "k_part_agg", "k_part_commit"]


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("khip::", "").replace("void ", "")
        name = re.sub(r"<.*", "", name).strip()
        per[name].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    n = int(sys.argv[3])
    cfg = sys.argv[5] if len(sys.argv) > 5 else "possible_fraud"
    hist = fetch.get("k_part_hist")
    factor = (16.0 * n) / (sum(hist) / len(hist)) if hist else 2.0
    per_kernel = {}
    total = 0.0
    for k in PUSH:
        if k not in fetch and k not in write:
            continue
        f = fetch.get(k, [0.0])
        w = write.get(k, [0.0])
        calls_per_push = 1 if k not in ("k_scan_excl",) else 1
        rd = factor * sum(f) / len(f)
        wr = sum(w) / len(w)
        per_kernel[k] = {"read_bytes": rd, "write_bytes": wr}
        total += (rd + wr) * calls_per_push
    out = {cfg: {"push": {"records": n, "hbm_bytes_per_launch": total, "fetch_calibration_factor": factor,
                          "per_kernel": per_kernel,
                          "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                                    "FETCH scaled by the k_part_hist calibration (16 B/record)"}}}
    try:
        prev = json.load(open(sys.argv[4]))
    except (OSError, ValueError):
        prev = {}
    prev.update(out)
    json.dump(prev, open(sys.argv[4], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
