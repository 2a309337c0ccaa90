"""Host-side cost of one C2 step's calls (reset, push, count_rows) with and without FLAG_PROFILE:
wall time of each call around a device-synchronised step, and the step's device time.  Diagnostic
for DESIGN.md §(e) (the bench's wall step vs its kernels' device time).
    python tools/host_overhead.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from ksql_amd import abi, synth  # noqa: E402


def main():
    lib = abi.load_product()
    n = 100_000_000
    card, ts = synth.possible_fraud(0, n, n, xp="torch", device="cuda")
    batch = abi.DeviceBatch(ts, keys=card)
    having = {"agg": 0, "op": "GT", "value": 3}
    for flags in (abi.FLAG_PROFILE, 0):
        h = abi.AggHandle(lib, abi.make_agg_desc(window_kind="TUMBLING", size_ms=5000, key_type="INT64",
                                                 aggs=[("COUNT_STAR", -1)], capacity_hint=30_000_000, flags=flags,
                                                 having=having))
        acc = {"reset": 0.0, "push": 0.0, "count": 0.0, "step": 0.0}
        steps = 20
        for i in range(steps + 3):
            t0 = time.perf_counter()
            h.reset()
            t1 = time.perf_counter()
            h.push(batch)
            t2 = time.perf_counter()
            h.count_rows(having)
            t3 = time.perf_counter()
            if i >= 3:
                acc["reset"] += t1 - t0
                acc["push"] += t2 - t1
                acc["count"] += t3 - t2
                acc["step"] += t3 - t0
        h.close()
        print("flags=%d: " % flags + " ".join("%s %.1f us" % (k, 1e6 * v / steps) for k, v in acc.items()), flush=True)


if __name__ == "__main__":
    main()
