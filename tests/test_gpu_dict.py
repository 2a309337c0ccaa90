"""The STRING-key dictionary (khip_dict.hpp) under forced fingerprint collisions.

Group identity is byte equality of the serialized key (GenericKeySerDe.java:95-117).
The dictionary compares a 22-bit hash fingerprint before the key bytes; two different keys that
share it meet on each other's slots: a row pending on a slot another row of its batch claimed is
resolved after the claims commit, and goes round again when the slot holds a different key.  The
tuning build's KHIP_DICT_FPMASK narrows the fingerprint (0: every key shares one) so that this
happens to every row, and KHIP_DICT_HASHMASK keeps the low 18 bits of the whole 64-bit key hash (keys
share full hashes: the same slot chain, fingerprint and hash word, told apart by their bytes
alone).  The UTF8 GROUP BY table (engines: partitioned, atomic) and a pull query (the read-only
probe) must still equal the oracle.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUNE_LIB = os.path.join(REPO, "ksql_amd", "libksqldb_hip_tune.so")


def _keys(rng, n, nkeys):
    # short (<= 8 B), 16-byte card numbers, and long (> 24 B) keys, incl. the empty string
    pool = [b"", b"x"] + [b"%016d" % (v * 7919) for v in range(nkeys // 2)] + \
           [b"k%05d" % v for v in range(nkeys // 4)] + [b"long-key-%040d" % v for v in range(nkeys // 4)]
    return [pool[i] for i in rng.integers(0, len(pool), n)]


def _check():
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from ksql_amd import abi
    from test_gpu_parity import assert_snap_equal
    from test_gpu_pull import _filter
    prod, orc = abi.load_product(), abi.load_oracle()
    assert prod.path.endswith("libksqldb_hip_tune.so"), prod.path
    rng = np.random.default_rng(5)
    for flags in (0, abi.FLAG_ENGINE_ATOMIC):
        kw = dict(window_kind="TUMBLING", size_ms=5000, key_type="UTF8", aggs=[("COUNT_STAR", -1)],
                  capacity_hint=1 << 20, flags=flags)
        gd, od = abi.make_agg_desc(**kw), abi.make_agg_desc(**kw)
        g, o = abi.AggHandle(prod, gd), abi.AggHandle(orc, od)
        t0 = 0
        for b in range(3):
            n = 200_000
            keys = _keys(rng, n, 40_000 * (b + 1))
            ts = t0 + (np.arange(n) * 20_000) // n
            t0 += 20_000
            batch = abi.HostBatch(ts, utf8_keys=keys)
            assert g.push(batch) == o.push(batch)
        osnap = o.snapshot()
        assert_snap_equal(g.snapshot(), osnap, gd)
        # pull query (the read-only probe) against the oracle's table filtered the same way
        probe = list(osnap["key"][::997][:100])
        probe.append(type(probe[0])("never-seen") if isinstance(probe[0], str) else b"never-seen")
        assert_snap_equal(g.get(keys=probe), _filter(osnap, probe, (None, None), (None, None), True), gd)
        g.close()
        o.close()
    print("OK")


@pytest.mark.parametrize("knobs", [{"KHIP_DICT_FPMASK": "0"}, {"KHIP_DICT_FPMASK": "1"}, {"KHIP_DICT_FPMASK": "255"},
                                   {"KHIP_DICT_HASHMASK": str(0x3FFFF)},
                                   {"KHIP_KEY_INLINE": "0", "KHIP_DICT_FPMASK": "0"}],
                         ids=lambda k: ",".join("%s=%s" % kv for kv in k.items()))
def test_dictionary_hash_collisions(knobs):
    if not os.path.exists(TUNE_LIB):
        pytest.skip("tuning build not present (make -C ksql_amd TUNING=1)")
    env = dict(os.environ, KSQL_AMD_LIB_VARIANT="tune", **knobs)
    p = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import test_gpu_dict as t; t._check()"
                        % os.path.join(REPO, "tests")], cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and p.stdout.strip().endswith("OK"), (p.stdout[-2000:], p.stderr[-3000:])


# Keys on both sides of the inline boundary (khip_dict.hpp): 0..17 ASCII digits are inline ids;
# 18+ digits, signs, spaces, a decimal point, full-width digits and letters are dictionary ids.
EDGE_KEYS = ["", "0", "00", "000", "7", "07", "007", "10", "12345678901234567", "99999999999999999",
             "00000000000000000", "01234567890123456", "123456789012345678", "000000000000000000",
             "1234567890123456789012", "12a", "a12", " 12", "12 ", "-12", "+12", "1.5", "\uff11\uff12", "x",
             "4000000000000000", "4000000000000001", "40000000000000010"]


@pytest.mark.parametrize("flags", [0, 2, 8], ids=["partitioned", "atomic", "changelog"])
def test_inline_and_dictionary_keys_vs_oracle(flags):
    from ksql_amd import abi
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from test_gpu_parity import assert_snap_equal
    from test_gpu_pull import _filter
    prod, orc = abi.load_product(), abi.load_oracle()
    rng = np.random.default_rng(11 + flags)
    kw = dict(window_kind="TUMBLING", size_ms=5000, key_type="UTF8", col_types=["INT64"],
              aggs=[("COUNT_STAR", -1), ("SUM", 0), ("MAX", 0)])
    gd, od = abi.make_agg_desc(**dict(kw, flags=flags)), abi.make_agg_desc(**kw)
    g, o = abi.AggHandle(prod, gd), abi.AggHandle(orc, od)
    t0 = 0
    for b in range(4):
        n = 30_000
        pool = EDGE_KEYS + ["%d" % v for v in rng.integers(0, 10**12, 500)] + ["k%d" % v for v in range(300)]
        keys = [pool[i] for i in rng.integers(0, len(pool), n)]
        ts = t0 + (np.arange(n) * 12_000) // n
        t0 += 9_000
        batch = abi.HostBatch(ts, utf8_keys=keys, cols=[rng.integers(-50, 50, n)])
        assert g.push(batch) == o.push(batch)
        if flags == 8:
            gc, oc = g.changes(), o.changes()
            assert_snap_equal(gc, oc, gd)
    osnap = o.snapshot()
    assert_snap_equal(g.snapshot(), osnap, gd)
    probe = EDGE_KEYS + ["12345", "never-seen", "5" * 17]
    assert_snap_equal(g.get(keys=probe), _filter(osnap, probe, (None, None), (None, None), True), gd)
    g.close()
    o.close()


def test_first_map_of_all_new_keys_grows_and_matches_oracle():
    """A first push of all-distinct dictionary keys outgrows the first map's table (sized for an
    eighth of the rows): the round is undone, the table grows for every probed row, and the map
    runs again; then a push of only inline keys, then dictionary keys again."""
    from ksql_amd import abi
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from test_gpu_parity import assert_snap_equal
    prod, orc = abi.load_product(), abi.load_oracle()
    kw = dict(window_kind="TUMBLING", size_ms=1000, key_type="UTF8", aggs=[("COUNT_STAR", -1)])
    gd = abi.make_agg_desc(**kw)
    g, o = abi.AggHandle(prod, gd), abi.AggHandle(orc, abi.make_agg_desc(**kw))
    n = 400_000
    for b, keys in enumerate((["key-%d" % v for v in range(n)], ["%d" % v for v in range(n)],
                              ["key-%d" % (v * 3) for v in range(n)])):
        batch = abi.HostBatch(np.full(n, 500 * b, np.int64), utf8_keys=keys)
        assert g.push(batch) == o.push(batch)
    assert_snap_equal(g.snapshot(), o.snapshot(), gd)
    g.close()
    o.close()
