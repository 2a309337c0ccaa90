"""Deterministic synthetic Kafka-shaped inputs for the BASELINE.json configs.

SURVEY.md §8(d) defines the shapes; this module fixes the exact formulas so the
same records can be generated on the host (numpy, for the CPU oracle / baseline
sample) and in HBM (torch on the GPU, for the bench and full-size tests) and
agree bit for bit.  All randomness is splitmix64 of (stream seed << 40) + index.

  C1 hourly_metrics   1e6 page_views, url = "http://ex.com/p/<id>", id ~ U[0, 1e4),
                      ts = 10 * i, COUNT(*) TUMBLING 1 HOUR GROUP BY url
  C2 possible_fraud   1e8 records, card_number = 4000000000000000 + id, id ~ U[0, 1e7),
                      ts = i * 10000 // n + U[0, 500), COUNT(*) TUMBLING 5 s, HAVING > 3
  C3 hopping_double   1e9 records, key ~ U[0, 1e5), value ~ U[0, 1000) with 1 % nulls,
                      ts = i * 3.6e6 // n + U[0, 1000), HOPPING 60 s / 10 s, GRACE 60 s,
                      SUM/AVG/MIN/MAX(value)
  C4 clickstream      users: user_id 1..1e8, level ~ U{Gold, Silver, Platinum} (codes 0..2);
                      clicks: 1e9, userid ~ U[1, 1.1e8], ts = i; LEFT JOIN ... WHERE
                      level = 'Platinum'
  C5 repartition_sum  1e9 records keyed by a random event id (source partition = event id % N),
                      region_id BIGINT ~ U[0, 1e6), amount BIGINT ~ U[-1e6, 1e6],
                      ts = i * 3.6e6 // n + U[0, 1000), GROUP BY region_id (non-key: repartition)
                      SUM(amount) TUMBLING 1 MINUTE
Weak scaling: rank r of N owns the keys k with k % N == r (key-hash sharding, the
Kafka-partition analogue); its records are generated from its own seed.
"""
import numpy as np

MASK64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
C1M = 0xBF58476D1CE4E5B9
C2M = 0x94D049BB133111EB
LEVELS = ["Gold", "Silver", "Platinum"]


def _s64(c):
    return c - (1 << 64) if c >= 1 << 63 else c


# ---------------------------------------------------------------- backends

class _Np:
    name = "numpy"

    @staticmethod
    def arange(lo, hi, device=None):
        return np.arange(lo, hi, dtype=np.uint64)

    @staticmethod
    def splitmix64(x):
        with np.errstate(over="ignore"):
            z = x + np.uint64(GOLDEN)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(C1M)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(C2M)
            return z ^ (z >> np.uint64(31))

    @staticmethod
    def u53(z):
        """top 53 bits as a non-negative int64."""
        return (z >> np.uint64(11)).astype(np.int64)

    @staticmethod
    def idx(lo, hi, device=None):
        return np.arange(lo, hi, dtype=np.int64)

    @staticmethod
    def to_f64(x):
        return x.astype(np.float64)


class _Torch:
    name = "torch"

    def __init__(self):
        import torch
        self.t = torch

    def arange(self, lo, hi, device=None):
        return self.t.arange(lo, hi, dtype=self.t.int64, device=device)

    def _srl(self, z, k):
        return (z >> k) & ((1 << (64 - k)) - 1)

    def splitmix64(self, x):
        z = x + _s64(GOLDEN)
        z = (z ^ self._srl(z, 30)) * _s64(C1M)
        z = (z ^ self._srl(z, 27)) * _s64(C2M)
        return z ^ self._srl(z, 31)

    def u53(self, z):
        return self._srl(z, 11)

    def idx(self, lo, hi, device=None):
        return self.t.arange(lo, hi, dtype=self.t.int64, device=device)

    def to_f64(self, x):
        return x.to(self.t.float64)


def backend(xp):
    if xp == "numpy" or xp is np:
        return _Np()
    return _Torch()


def _stream(be, seed, lo, hi, device, sub=0, nsub=1):
    """splitmix64 values for indices [lo, hi) of stream `seed` (interleaved sub-streams)."""
    base = (seed << 40)
    x = be.arange(lo, hi, device) if be.name == "torch" else be.arange(lo, hi)
    if be.name == "numpy":
        x = x * np.uint64(nsub) + np.uint64(base + sub)
    else:
        x = x * nsub + (base + sub)
    return be.splitmix64(x)


# ---------------------------------------------------------------- configs

CONFIGS = {
    "hourly_metrics": dict(n=1_000_000, keys=10_000, seed=1, size_ms=3_600_000),
    "possible_fraud": dict(n=100_000_000, keys=10_000_000, seed=2, span_ms=10_000, disorder_ms=500,
                           size_ms=5_000, having_gt=3),
    "hopping_double": dict(n=1_000_000_000, keys=100_000, seed=3, span_ms=3_600_000, disorder_ms=1_000,
                           size_ms=60_000, advance_ms=10_000, grace_ms=60_000, null_pct=1),
    "clickstream_join": dict(users=100_000_000, n=1_000_000_000, seed_users=4, seed_clicks=5,
                             miss_factor=1.1),
    "repartition_sum": dict(n=1_000_000_000, regions=1_000_000, seed=6, span_ms=3_600_000, disorder_ms=1_000,
                            size_ms=60_000),
}


def possible_fraud(lo, hi, n, xp="numpy", device=None, rank=0, world=1, keys=10_000_000, seed=2,
                   span_ms=10_000, disorder_ms=500):
    """Records [lo, hi) of a run of n records: (card BIGINT key, ts)."""
    be = backend(xp)
    s = seed + 1000 * rank
    z = _stream(be, s, lo, hi, device, 0, 2)
    kid = be.u53(z) % keys
    card = (kid * world + rank) + 4_000_000_000_000_000
    i = be.idx(lo, hi, device)
    d = be.u53(_stream(be, s, lo, hi, device, 1, 2)) % disorder_ms
    ts = (i * span_ms) // n + d
    return card, ts


URL_PREFIX = b"http://ex.com/p/"


def hourly_metrics(lo, hi, n=1_000_000, keys=10_000, seed=1):
    """C1 (host only): (url strings, ts)."""
    be = _Np()
    kid = be.u53(_stream(be, seed, lo, hi, None)) % keys
    ts = np.arange(lo, hi, dtype=np.int64) * 10
    urls = ["http://ex.com/p/%d" % k for k in kid.tolist()]
    return urls, ts


def hourly_metrics_utf8(lo, hi, n=1_000_000, keys=10_000, seed=1):
    """C1 as a columnar UTF-8 key column: (key_offsets int64[m+1], key_bytes uint8, ts), the
    same urls as hourly_metrics(), built without Python strings."""
    be = _Np()
    kid = be.u53(_stream(be, seed, lo, hi, None)) % keys
    ts = np.arange(lo, hi, dtype=np.int64) * 10
    nd = np.ones(len(kid), np.int64)
    for p in (10, 100, 1000, 10_000, 100_000):
        nd += (kid >= p)
    lens = len(URL_PREFIX) + nd
    offs = np.zeros(len(kid) + 1, np.int64)
    offs[1:] = np.cumsum(lens)
    out = np.empty(int(offs[-1]), np.uint8)
    pre = np.frombuffer(URL_PREFIX, np.uint8)
    for j in range(len(pre)):
        out[offs[:-1] + j] = pre[j]
    for j in range(int(nd.max()) if len(nd) else 0):  # digit j from the left
        has = nd > j
        d = (kid[has] // (10 ** (nd[has] - 1 - j))) % 10
        out[offs[:-1][has] + len(pre) + j] = (d + 48).astype(np.uint8)
    return offs, out, ts


def card_utf8(card, xp="numpy"):
    """16-digit card numbers (int64 4000000000000000 + id) → UTF-8 key column
    (key_offsets [n+1], key_bytes [16 n]): the VARCHAR card_number of possible_fraud."""
    if xp == "numpy" or xp is np:
        p10 = 10 ** np.arange(15, -1, -1, dtype=np.int64)
        digits = ((card[:, None] // p10[None, :]) % 10 + 48).astype(np.uint8).reshape(-1)
        offs = np.arange(len(card) + 1, dtype=np.int64) * 16
        return offs, digits
    import torch
    p10 = torch.tensor([10 ** k for k in range(15, -1, -1)], dtype=torch.int64, device=card.device)
    digits = ((card[:, None] // p10[None, :]) % 10 + 48).to(torch.uint8).reshape(-1)
    offs = torch.arange(card.numel() + 1, dtype=torch.int64, device=card.device) * 16
    return offs, digits


def hopping_double(lo, hi, n, xp="numpy", device=None, rank=0, world=1, keys=100_000, seed=3,
                   span_ms=3_600_000, disorder_ms=1_000, null_pct=1):
    """(key BIGINT, ts, value DOUBLE, value_valid bool)."""
    be = backend(xp)
    s = seed + 1000 * rank
    k = be.u53(_stream(be, s, lo, hi, device, 0, 4)) % keys
    key = k * world + rank
    i = be.idx(lo, hi, device)
    ts = (i * span_ms) // n + be.u53(_stream(be, s, lo, hi, device, 1, 4)) % disorder_ms
    val = be.to_f64(be.u53(_stream(be, s, lo, hi, device, 2, 4))) * (2.0 ** -53) * 1000.0
    valid = (be.u53(_stream(be, s, lo, hi, device, 3, 4)) % 100) >= null_pct
    return key, ts, val, valid


def users_table(lo, hi, xp="numpy", device=None, seed_users=4):
    """user_id = i + 1, level code ~ U{0,1,2}."""
    be = backend(xp)
    uid = be.idx(lo + 1, hi + 1, device)
    level = be.u53(_stream(be, seed_users, lo, hi, device)) % 3
    return uid, level


def clicks(lo, hi, users, xp="numpy", device=None, seed_clicks=5, miss_factor=1.1):
    be = backend(xp)
    span = int(users * miss_factor)
    uid = be.u53(_stream(be, seed_clicks, lo, hi, device)) % span + 1
    ts = be.idx(lo, hi, device)
    return uid, ts


SPARSE_MULT = 0x9E3779B97F4A7C15  # odd: id -> id * M mod 2^40 is a bijection of [0, 2^40)


def sparse_ids(uid):
    """User ids 1..U spread over [0, 2^40) (clickstream_join --sparse-ids): no dense index."""
    if hasattr(uid, "dtype") and str(uid.dtype).startswith("torch"):
        import torch
        m = torch.tensor(SPARSE_MULT - (1 << 64), dtype=torch.int64, device=uid.device)  # wraps like uint64
        return (uid * m) & ((1 << 40) - 1)
    import numpy as np
    with np.errstate(over="ignore"):
        return ((np.asarray(uid, np.uint64) * np.uint64(SPARSE_MULT)) & np.uint64((1 << 40) - 1)).astype(np.int64)


def repartition_sum(lo, hi, n, xp="numpy", device=None, rank=0, world=1, regions=1_000_000, seed=6,
                    span_ms=3_600_000, disorder_ms=1_000):
    """C5 source partition `rank`: (event_id key, ts, region_id BIGINT, amount BIGINT)."""
    be = backend(xp)
    s = seed + 1000 * rank
    eid = (be.u53(_stream(be, s, lo, hi, device, 0, 4)) >> 8) * world + rank
    i = be.idx(lo, hi, device)
    ts = (i * span_ms) // n + be.u53(_stream(be, s, lo, hi, device, 1, 4)) % disorder_ms
    region = be.u53(_stream(be, s, lo, hi, device, 2, 4)) % regions
    amount = be.u53(_stream(be, s, lo, hi, device, 3, 4)) % 2_000_001 - 1_000_000
    return eid, ts, region, amount
