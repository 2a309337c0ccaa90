"""Single-process timing of the repartition pack (khip_shuffle_pack / khip_shuffle_pack_v) on C5's
records, for 1..8 destinations: the pack kernel alone, without the other ranks of a one-device
rehearsal competing for the GPU.  Wall time around the call (pack_v returns its counts, so the
call ends synchronised); bytes = the algorithmic 24 B read + row_words x 8 B written per record.
    python tools/pack_bench.py [--records N] [--reps R]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=125_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--parts", default="1,2,4,8")
    a = ap.parse_args()
    import torch
    from ksql_amd import abi, synth
    lib = abi.load_product()
    n = a.records
    eid, ts, region, amount = synth.repartition_sum(0, n, n, xp="torch", device="cuda", rank=0, world=1)
    src = abi.DeviceBatch(ts, cols=[region, amount])
    torch.cuda.synchronize()
    for P in [int(x) for x in a.parts.split(",")]:
        sh = abi.ShuffleHandle(lib, P, 0, ["INT64", "INT64"], 0)
        send = torch.empty((sh.pack_capacity(n), sh.row_words), dtype=torch.int64, device="cuda")
        fn = (lambda: sh.pack(src, send=send)) if P == 1 else (lambda: sh.pack_v(src, send=send))
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        by = n * (24 + 8 * sh.row_words)
        print(json.dumps({"parts": P, "records": n, "row_words": sh.row_words, "ms": best * 1e3,
                          "GBps": by / best / 1e9}), flush=True)
        del send
        sh.close()


if __name__ == "__main__":
    main()
