"""The partitioned engine's alternative kernel paths, forced through the tuning build's knobs.

The release library always takes the measured defaults, so some paths run only when a push
declines the default one.  Here each knob set runs in a child process on the tuning build
(`KSQL_AMD_LIB_VARIANT=tune`: the same kernels, KHIP_* knobs read from the environment), with a
COUNT(*) TUMBLING + HAVING workload against the oracle (table, batch statistics, HAVING count):
- KHIP_C1P=0: the general path instead of the COUNT(*) pipeline (khip_agg_c1.hip);
- KHIP_R8K=0: R8 records through the general scatter / refine kernels, not their own ones;
- KHIP_R8_U=4: R8 staged steps of 4 records per thread;
- KHIP_SCATTER2=0: one-level scatter (no refine pass);
- KHIP_R8=0: 12-byte (R12) records where R8 would fit;
- KHIP_C1P=0 + KHIP_C1_AU=4: the general path's COUNT(*) merge with fewer records per thread;
- KHIP_C1_LOG2H=13 / 11: the pipeline's merge with a twice larger LDS table, and with a twice
  smaller one (partitions overflow it: the sub-pass retries);
- KHIP_C1V=0: value aggregates through the general path instead of the value-record pipeline;
  KHIP_C1V_SPEC=0: its merge without the plane-shape specialisation (SUM(BIGINT) here);
  KHIP_C1V_LOG2H=9: a small LDS table (sub-pass retries, split by key).
Each case runs COUNT(*) TUMBLING + HAVING and SUM of a BIGINT + HAVING over HOPPING (panes).
Dense and sparse key ranges, several pushes (resident rows), late records (the pipeline declines).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUNE_LIB = os.path.join(REPO, "ksql_amd", "libksqldb_hip_tune.so")

KNOBS = [
    {"KHIP_C1P": "0"},
    {"KHIP_C1P": "0", "KHIP_R8K": "0"},
    {"KHIP_C1P": "0", "KHIP_R8_U": "4"},
    {"KHIP_C1P": "0", "KHIP_SCATTER2": "0"},
    {"KHIP_C1P": "0", "KHIP_R8": "0"},
    {"KHIP_C1P": "0", "KHIP_C1_AU": "4"},
    {"KHIP_C1_LOG2H": "13"},
    {"KHIP_C1_LOG2H": "11"},
    {"KHIP_C1V": "0"},
    {"KHIP_C1V_SPEC": "0"},
    {"KHIP_C1V_LOG2H": "9"},
]


def _check():
    """Child process: every case against the oracle; prints OK."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from ksql_amd import abi
    from test_gpu_parity import assert_snap_equal
    prod, orc = abi.load_product(), abi.load_oracle()
    assert prod.path.endswith("libksqldb_hip_tune.so"), prod.path
    having = {"agg": 0, "op": "GT", "value": 2}
    for case in ("dense", "sparse", "late"):
        rng = np.random.default_rng(len(case))
        batches = []
        t0 = 0
        for b in range(3):
            n = 600_000
            if case == "sparse":
                k = rng.integers(0, 50_000, n) * 7919 + (1 << 45)
            else:
                k = rng.integers(0, 50_000, n)
            ts = t0 + (np.arange(n) * 20_000) // n + rng.integers(0, 400, n)
            if case == "late":
                ts[rng.random(n) < 0.02] -= 15_000
            t0 += 20_000
            v = rng.integers(-1000, 1000, n)
            batches.append(abi.HostBatch(ts, keys=k, cols=[v], col_valid=[rng.random(n) > 0.02]))
        grace = 2000 if case == "late" else -1
        kws = [dict(window_kind="TUMBLING", size_ms=5000, grace_ms=grace, aggs=[("COUNT_STAR", -1)], having=having,
                    capacity_hint=1 << 22),
               dict(window_kind="HOPPING", size_ms=6000, advance_ms=2000, grace_ms=grace, col_types=["INT64"],
                    aggs=[("SUM", 0)], having={"agg": 0, "op": "GT", "value": 0},
                    capacity_hint=1 << 22)]
        for kw in kws:
            gd, od = abi.make_agg_desc(**kw), abi.make_agg_desc(**kw)
            g, o = abi.AggHandle(prod, gd), abi.AggHandle(orc, od)
            for b in batches:
                gs, os_ = g.push(b), o.push(b)
                assert gs == os_, (case, gs, os_)
            assert_snap_equal(g.snapshot(), o.snapshot(), gd)
            assert g.count_rows(kw["having"]) == o.snapshot(kw["having"])["n"], case
            g.close()
            o.close()
    print("OK")


@pytest.mark.parametrize("knobs", KNOBS, ids=lambda k: ",".join("%s=%s" % kv for kv in k.items()))
def test_knob_paths_match_oracle(knobs):
    if not os.path.exists(TUNE_LIB):
        pytest.skip("tuning build not present (make -C ksql_amd TUNING=1)")
    env = dict(os.environ, KSQL_AMD_LIB_VARIANT="tune", **knobs)
    p = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import test_gpu_knobs as t; t._check()"
                        % os.path.join(REPO, "tests")], cwd=REPO, env=env, capture_output=True, text=True, timeout=200)
    assert p.returncode == 0 and p.stdout.strip().endswith("OK"), (p.stdout[-2000:], p.stderr[-3000:])
