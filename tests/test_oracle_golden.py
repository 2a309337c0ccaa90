"""The CPU oracle (test infrastructure) against the reference's own QTT golden
vectors: this is what pins the oracle before it is trusted as the parity checker."""
import pytest

import qtt
from ksql_amd import abi

AGG_CASES = qtt.load_cases("agg")
JOIN_CASES = qtt.load_cases("join")


@pytest.fixture(scope="module")
def orc():
    return abi.load_oracle()


def test_fixture_inventory():
    # the hot-path goldens named in SURVEY.md §4 / §8(c) are all present
    srcs = {c["source"] for c in AGG_CASES} | {c["source"] for c in JOIN_CASES}
    for s in ["tumbling-windows.json:7", "tumbling-windows.json:45", "tumbling-windows.json:71",
              "hopping-windows.json:7", "hopping-windows.json:50", "hopping-windows.json:80",
              "hopping-windows.json:135", "count.json:7", "sum.json:7", "sum.json:55", "sum.json:74",
              "average-udaf.json:7", "average-udaf.json:32", "average-udaf.json:57", "min-group-by.json:41",
              "min-group-by.json:70", "max-group-by.json:12", "max-group-by.json:43", "max-group-by.json:74",
              "having.json:7", "window-bounds.json:31", "window-bounds.json:56", "group-by.json:79",
              "null.json:70", "joins.json:1530", "joins.json:1594"]:
        assert s in srcs, s


@pytest.mark.parametrize("split", [None, 1, 2])
@pytest.mark.parametrize("case", AGG_CASES, ids=["%s %s" % (c["source"], c["name"]) for c in AGG_CASES])
def test_oracle_aggregate_golden(orc, case, split):
    assert qtt.compare_agg(case, qtt.run_agg_case(orc, case, split)) == []


@pytest.mark.parametrize("case", AGG_CASES, ids=["%s %s" % (c["source"], c["name"]) for c in AGG_CASES])
def test_oracle_output_sequence_golden(orc, case):
    """Every output record the reference emits, in order: pushes of one record each are the
    reference's cache-off, emit-at-every-record run (HAVING tombstones, EMIT FINAL)."""
    assert qtt.compare_outputs(case, qtt.run_agg_outputs(orc, case, 1)) == []


@pytest.mark.parametrize("case", JOIN_CASES, ids=["%s %s" % (c["source"], c["name"]) for c in JOIN_CASES])
def test_oracle_join_golden(orc, case):
    assert qtt.compare_join(case, qtt.run_join_case(orc, case)) == []


def test_oracle_detects_a_wrong_answer(orc):
    # the comparator is not vacuous: perturb an expected value and it must fail
    import copy
    case = copy.deepcopy(next(c for c in AGG_CASES if c["source"] == "hopping-windows.json:135"))
    case["expected"][0]["values"][0] += 1
    assert qtt.compare_agg(case, qtt.run_agg_case(orc, case)) != []
