"""Synthetic generators: deterministic, host (numpy) == device-form (torch) bit for bit,
and shaped as SURVEY.md §8(d) says."""
import numpy as np
import pytest

from ksql_amd import synth


def test_possible_fraud_numpy_equals_torch():
    torch = pytest.importorskip("torch")
    a = synth.possible_fraud(5, 20005, 10**8)
    b = synth.possible_fraud(5, 20005, 10**8, xp="torch")
    assert np.array_equal(a[0], b[0].numpy()) and np.array_equal(a[1], b[1].numpy())


def test_hopping_numpy_equals_torch():
    pytest.importorskip("torch")
    a = synth.hopping_double(0, 10000, 10**9)
    b = synth.hopping_double(0, 10000, 10**9, xp="torch")
    for x, y in zip(a, b):
        assert np.array_equal(x, y.numpy())


def test_possible_fraud_shape():
    n = 200_000
    card, ts = synth.possible_fraud(0, n, n, keys=10_000)
    assert card.min() >= 4_000_000_000_000_000 and card.max() < 4_000_000_000_010_000
    assert ts.min() >= 0 and ts.max() < 10_000 + 500
    # prefix property used by the CPU baseline sample
    c2, t2 = synth.possible_fraud(0, 1000, n, keys=10_000)
    assert np.array_equal(card[:1000], c2) and np.array_equal(ts[:1000], t2)


def test_weak_scaling_shards_are_disjoint():
    n = 10_000
    shards = [synth.possible_fraud(0, n, n, rank=r, world=4, keys=1000)[0] for r in range(4)]
    for r, s in enumerate(shards):
        assert ((s - 4_000_000_000_000_000) % 4 == r).all()
