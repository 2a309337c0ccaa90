"""Debug: test_gpu_c1.py::test_c1_declined_pushes[ts_span] (stream_time mismatch in r04g)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from ksql_amd import abi  # noqa: E402

prod, orc = abi.load_product(), abi.load_oracle()
print("lib", prod.path)
rng = np.random.default_rng(7)
n = 400_000
k = rng.integers(0, 30_000, n)
ts = (np.arange(n) * 10_000) // n + rng.integers(0, 500, n)
ts[-1000:] += 1 << 32
for lib, name in ((prod, "prod"), (orc, "oracle")):
    d = abi.make_agg_desc(window_kind="TUMBLING", size_ms=5000, advance_ms=5000, grace_ms=-1,
                          aggs=[("COUNT_STAR", -1)], capacity_hint=1 << 22,
                          flags=abi.FLAG_PROFILE if lib is prod else 0,
                          having={"agg": 0, "op": "GT", "value": 3})
    h = abi.AggHandle(lib, d)
    st = h.push(abi.HostBatch(ts, keys=k))
    print(name, st)
    if lib is prod:
        kt = h.kernel_times()
        print("kt", {x: kt[x] for x in kt if "c1" in x})
    h.close()
