"""The partitioned engine's record formats (khip_agg_part.hip, k_part_wrange): a push whose key
range and event-time span fit one 64-bit word together travels as 8-byte records ((key - kbase)
<< tb | rowtime delta, R8); otherwise as 12-byte (key hash, rowtime delta) records (R12).  Both
formats, and the boundary between them, against the oracle: COUNT(*) TUMBLING with HAVING (the
lean merge), BIGINT keys over ranges of 2^8 .. 2^64 and event-time spans of 2^10 .. 2^30 ms, late
records and several pushes (resident rows merged with new ones)."""
import numpy as np
import pytest

from ksql_amd import abi
from test_gpu_parity import assert_snap_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def prod():
    return abi.load_product()


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def _push_all(lib, desc, batches):
    h = abi.AggHandle(lib, desc)
    stats = [h.push(b) for b in batches]
    snap = h.snapshot(desc_having(desc))
    n = h.count_rows(desc_having(desc)) if lib.product else snap["n"]  # the maintained HAVING count
    h.close()
    return stats, snap, n


def desc_having(desc):
    return {"agg": 0, "op": "GT", "value": 1}


@pytest.mark.parametrize("kbits", [8, 24, 40, 54, 64])
@pytest.mark.parametrize("tbits", [10, 20, 30])
def test_r8_r12_boundary(prod, orc, kbits, tbits):
    rng = np.random.default_rng(kbits * 100 + tbits)
    n = 200_000
    nkeys = 4000
    if kbits == 64:
        pool = rng.integers(-2**63, 2**63 - 1, nkeys, dtype=np.int64)
        pool[:2] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max]
    else:
        base = int(rng.integers(-2**62, 2**62))
        pool = base + rng.integers(0, 2**kbits, nkeys, dtype=np.int64)
        pool[:2] = [base, base + 2**kbits - 1]
    span = 2**tbits
    batches = []
    t0 = int(rng.integers(0, 2**40))
    for b in range(3):
        keys = pool[rng.integers(0, nkeys, n)]
        ts = t0 + np.sort(rng.integers(0, span, n)) + rng.integers(0, max(span // 50, 1), n)
        ts[rng.random(n) < 0.001] -= span  # a few late records
        kv = rng.random(n) > 0.01
        batches.append(abi.HostBatch(ts, keys=keys, key_valid=kv))
        t0 += span // 2
    size = max(span // 16, 1000)
    kw = dict(window_kind="TUMBLING", size_ms=size, advance_ms=size, grace_ms=size, aggs=[("COUNT_STAR", -1)],
              having=desc_having(None))
    gd, od = abi.make_agg_desc(**kw), abi.make_agg_desc(**kw)
    gs, g, gn = _push_all(prod, gd, batches)
    os_, o, on = _push_all(orc, od, batches)
    assert gs == os_
    assert gn == on
    assert_snap_equal(g, o, gd)
