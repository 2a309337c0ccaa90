#!/usr/bin/env python3
"""HBM traffic per bench step from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs).

The profiled command is `bench.py --config <leg> --steps S --warmup W --no-cpu-baseline
--no-extras`: every library dispatch of the run belongs to one of the S + W identical steps
(the generators and the copy-rate probe are torch kernels and are excluded by name), so
bytes per step = sum over the library's dispatches / (S + W).

Units and the gfx950 correction (MI355X_MICROARCH.md:297-299, HBM / rocprofv3): FETCH_SIZE and
WRITE_SIZE are in KB; FETCH_SIZE reports 1/2 of the bytes of a wide coalesced streaming read
(16 B per lane), so the reads of the STREAMING kernels below are doubled.  Every other kernel's
reads (random gathers: hash-probe slots, dense-index cells, dictionary / source-table rows, serde
byte loads) are reported raw, labelled "gather": the correction is not established for them, and
FETCH_SIZE counts L2 → fabric requests, Infinity-Cache (MALL) hits included, so their figure is
L2-miss bytes, not HBM bytes.  WRITE_SIZE is taken as reported.  Where the run contains
k_part_hist, whose reads are exactly 16 B x records (key + ts) per step, the measured factor
(true bytes / raw FETCH bytes, per step) is reported beside the 2.0 as a check.

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


# wide coalesced streaming readers (16-B-per-lane loads of contiguous runs): FETCH_SIZE x 2
STREAMING = ("k_part_hist", "k_part_scatter", "k_part_scatter_r8", "k_part_scatter_w", "k_part_refine", "k_part_refine_r8", "k_part_merge", "k_part_merge_c1", "k_part_agg",
             "k_part_colsum", "k_part_colbase", "k_part_colprefix", "k_part_pscan", "k_scan_blocks", "k_part_rows",
             "k_part_chg", "k_part_stats", "k_part_wrange", "k_part_commit", "k_part_reset", "k_part_tsrange",
             "k_shuf_hist", "k_shuf_pack", "k_shuf_unpack", "k_shuf_colsum", "k_shuf_prefix", "k_init_table")


def fetch_factor(name):
    return 2.0 if name in STREAMING else 1.0


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
    gather = 0.0
    for k in sorted(set(fetch) | set(write)):
        f = fetch_factor(k)
        rd = f * sum(fetch.get(k, [])) / steps
        wr = sum(write.get(k, [])) / steps
        per_kernel[k] = {"read_bytes_per_step": rd, "write_bytes_per_step": wr, "fetch_factor": f,
                         "read_class": "stream" if f == 2.0 else "gather (raw L2->fabric bytes, MALL hits included)",
                         "dispatches_per_step": len(fetch.get(k, write.get(k, []))) / steps}
        total += rd + wr
        if f != 2.0:
            gather += rd
    rec = {"records": n, "hbm_bytes_per_step": total, "hbm_bytes_per_record": total / n,
           "gather_read_bytes_per_step": gather, "per_kernel": per_kernel,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over the same bench "
                     "command; library kernels only; FETCH_SIZE x 2 for the streaming kernels (gfx950 "
                     "wide-stream correction), x 1 (raw) for gathers"}
    hist = fetch.get("k_part_hist")
    if hist:  # true / raw, per step: 16 B x records of key + ts per step over the raw bytes per step
        rec["k_part_hist_fetch_factor_measured"] = (16.0 * n) / (sum(hist) / steps)
    try:
        prev = json.load(open(out_path))
    except (OSError, ValueError):
        prev = {}
    prev[cfg] = rec
    json.dump(prev, open(out_path, "w"), indent=1)
    print(json.dumps({cfg: {k: v for k, v in rec.items() if k != "per_kernel"}}, indent=1))


if __name__ == "__main__":
    main()
