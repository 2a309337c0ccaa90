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
                                   {"KHIP_DICT_HASHMASK": str(0x3FFFF)}],
                         ids=lambda k: ",".join("%s=%s" % kv for kv in k.items()))
def test_dictionary_hash_collisions(knobs):
    if not os.path.exists(TUNE_LIB):
        pytest.skip("tuning build not present (make -C ksql_amd TUNING=1)")
    env = dict(os.environ, KSQL_AMD_LIB_VARIANT="tune", **knobs)
    p = subprocess.run([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import test_gpu_dict as t; t._check()"
                        % os.path.join(REPO, "tests")], cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0 and p.stdout.strip().endswith("OK"), (p.stdout[-2000:], p.stderr[-3000:])
