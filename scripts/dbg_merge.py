import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch; torch.cuda.init()
import numpy as np
import qtt
from ksql_amd import abi
lib = abi.load_product()
case = [c for c in qtt.load_cases("agg") if c["name"] == "average int"][0]
print(case["desc"])
print([ (r["key"], r["cols"], r["ts"]) for r in case["input"]])
snap = qtt.run_agg_case(lib, case, None)
print({k: snap[k] for k in ("n", "key", "ws", "rowtime", "values", "nulls")})
print(case["expected"])
