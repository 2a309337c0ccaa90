#!/bin/bash
# Round 5: dictionary rework tests + utf8 leg, then merge variant A/Bs (build_variant.sh libraries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_time_domains.py \
  tests/test_gpu_c1.py tests/test_gpu_join_string.py tests/test_gpu_pull.py tests/test_gpu_parity.py \
  "tests/test_gpu_fullsize.py::test_c2_possible_fraud_utf8_full" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "^FAILED" $O/tests.log | head -20; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python3 bench.py --utf8 --steps 5 --no-cpu-baseline --no-extras > $O/utf8.jsonl 2> $O/utf8.err || exit 4
cut -c1-250 $O/utf8.jsonl
VARIANTS="rel defer nolist" KGREP="k_c1_merge|k_c1_scatter|k_c1_refine" bash scripts/ab_bench.sh r05e_c2 2 || exit 5
VARIANTS="rel condmm" KGREP="k_c1v_merge" BENCH_ARGS="--config hopping_double --steps 1 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r05e_c3 1 || exit 6
VARIANTS="rel defer condmm" KGREP="k_c1v_merge" BENCH_ARGS="--config repartition_sum --steps 3 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r05e_c5 1 || exit 7
