#!/usr/bin/env python3
"""HBM traffic per bench step from rocprofv3 counter passes (separate runs of the same command).

The profiled command is `bench.py --config <leg> --steps S --warmup W --no-cpu-baseline
--no-extras`: every library dispatch of the run belongs to one of the S + W identical steps (the
generators and the copy-rate probe are torch kernels and are excluded by name), so bytes per step
= sum over the library's dispatches / (S + W).

Read bytes are MEASURED per dispatch from the L2's memory-side read requests by size, collected in
one pass: TCC_EA0_RDREQ_32B_sum x 32 + TCC_EA0_RDREQ_64B_sum x 64 + TCC_EA0_RDREQ_128B_sum x 128.
No kernel list decides a correction.  The derived FETCH_SIZE (its own pass) is kept beside it as
`fetch_size_raw`: on gfx950 FETCH_SIZE tallies a 128-B request at 64 B (MI355X_MICROARCH.md, HBM /
rocprofv3: "FETCH_SIZE reports exactly 1/2 of the bytes of a wide coalesced streaming read"), so
for a streaming kernel read_bytes ≈ 2 x fetch_size_raw, for a gather of 32/64-B lines ≈ 1 x.
Round 4 applied the x 2 from a hand-kept list of kernel names, which went stale as kernels were
added; the size-classed count cannot.  Request bytes count L2 -> fabric
traffic, Infinity-Cache (MALL) hits included: for a gather whose table is MALL-resident they are
L2-miss bytes, not HBM bytes.  WRITE_SIZE (own pass) is taken as reported.

usage: pmc_traffic.py <rdreq csv> <fetch csv | -> <write csv> <records> <steps incl. warmup>
                      <out json> <config key>
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

REQ_BYTES = {"TCC_EA0_RDREQ_32B_sum": 32.0, "TCC_EA0_RDREQ_64B_sum": 64.0, "TCC_EA0_RDREQ_128B_sum": 128.0,
             "TCC_EA0_RDREQ_32B": 32.0, "TCC_EA0_RDREQ_64B": 64.0, "TCC_EA0_RDREQ_128B": 128.0}


def library_kernel(name):
    # the library's kernels (torch's are at::native::...), minus the setup ones
    return name.startswith("k_") and name not in OUTSIDE_STEP


def load(path, counters, scale):
    """{kernel: {dispatch id: bytes}} summed over the given counters (x their scale)."""
    per = defaultdict(lambda: defaultdict(float))
    if path in (None, "-"):
        return per
    for r in csv.DictReader(open(path)):
        c = r["Counter_Name"]
        if c not in counters:
            continue
        name = kname(r["Kernel_Name"])
        if library_kernel(name):
            per[name][r["Dispatch_Id"]] += float(r["Counter_Value"]) * scale(c)
    return per


def summarize(rdreq, fetch, write, n, steps):
    per_kernel = {}
    total = 0.0
    for k in sorted(set(rdreq) | set(write)):
        rd = sum(rdreq.get(k, {}).values()) / steps
        wr = sum(write.get(k, {}).values()) / steps
        fs = sum(fetch.get(k, {}).values()) / steps if k in fetch else None
        d = {"read_bytes_per_step": rd, "write_bytes_per_step": wr,
             "dispatches_per_step": len(rdreq.get(k, write.get(k, {}))) / steps}
        if fs is not None:
            d["fetch_size_raw_per_step"] = fs
            d["read_over_fetch_size"] = rd / fs if fs > 0 else None
        per_kernel[k] = d
        total += rd + wr
    return {"records": n, "method_version": 2, "hbm_bytes_per_step": total, "hbm_bytes_per_record": total / n,
            "per_kernel": per_kernel,
            "method": "rocprofv3 passes over the same bench command: TCC_EA0_RDREQ_{32B,64B,128B}_sum (read "
                      "requests by size, bytes = count x size), WRITE_SIZE, and FETCH_SIZE as a cross-check "
                      "(fetch_size_raw); library kernels only; per step = sum / (steps + warmup)"}


def main():
    rdreq = load(sys.argv[1], REQ_BYTES, lambda c: REQ_BYTES[c])
    fetch = load(sys.argv[2], ("FETCH_SIZE",), lambda c: 1024.0)
    write = load(sys.argv[3], ("WRITE_SIZE",), lambda c: 1024.0)
    n = int(sys.argv[4])
    steps = int(sys.argv[5])
    out_path, cfg = sys.argv[6], sys.argv[7]
    if not rdreq:
        sys.exit("no TCC_EA0_RDREQ_*B rows for library kernels in %s" % sys.argv[1])
    rec = summarize(rdreq, fetch, write, n, steps)
    try:
        prev = json.load(open(out_path))
    except (OSError, ValueError):
        prev = {}
    prev[cfg] = rec
    json.dump(prev, open(out_path, "w"), indent=1)
    print(json.dumps({cfg: {k: v for k, v in rec.items() if k != "per_kernel"}}, indent=1))
    for k, d in sorted(rec["per_kernel"].items(), key=lambda kv: -kv[1]["read_bytes_per_step"])[:12]:
        print("%-28s read %8.1f MB  write %8.1f MB  read/FETCH_SIZE %s" % (
            k, d["read_bytes_per_step"] / 1e6, d["write_bytes_per_step"] / 1e6,
            "%.2f" % d["read_over_fetch_size"] if d.get("read_over_fetch_size") else "-"))


if __name__ == "__main__":
    main()
