import os, sys, json
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np
from ksql_amd import abi
import qtt
cases = [c for c in qtt.load_cases("agg") if "grace is specified as zero" in c["name"] and c["source"].startswith("suppress")]
case = cases[0]
lib = abi.load_product()
d = case["desc"]
h = abi.AggHandle(lib, qtt.case_desc(case))
for lo in range(len(case["input"])):
    b = qtt.case_batch(case, lo, lo + 1)
    st = h.push(b)
    s = h.snapshot(None)
    print("push", lo, {k: st[k] for k in ("rows_accepted", "windows_applied", "windows_late", "stream_time")},
          [(s["key"][i], int(s["ws"][i]), int(s["rowtime"][i]), int(s["values"][0][i])) for i in range(s["n"])], flush=True)
h.close()
