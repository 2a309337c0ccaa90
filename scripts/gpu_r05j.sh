#!/bin/bash
# Round 5: inline ids (no hash, no list append, no resolve pass without pending rows) — parity, C2 --utf8 both ways,
# joins, pull queries, C2 --utf8 at full size), the C2 --utf8 leg both ways, its traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -x --timeout 600 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_parity.py \
  tests/test_gpu_join_string.py tests/test_gpu_emit.py tests/test_gpu_pull.py tests/test_gpu_c1.py \
  "tests/test_gpu_fullsize.py::test_c2_possible_fraud_utf8_full" "tests/test_gpu_fullsize.py::test_c1_hourly_metrics_full" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for F in digits alnum; do
  timeout -k 10 300 python3 bench.py --utf8 --card-format $F --steps 10 --warmup 3 --no-cpu-baseline > $O/utf8_$F.jsonl 2> $O/utf8_$F.err || { tail $O/utf8_$F.err; exit 4; }
  cut -c1-260 $O/utf8_$F.jsonl
done
STEPS=3 bash scripts/profile_leg.sh r05j possible_fraud --utf8 > $O/prof_utf8.log 2>&1 || { tail -8 $O/prof_utf8.log; exit 7; }
head -16 $O/prof_utf8.log
BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-extras" KFILT="k_c1_(merge|scatter|refine)" bash scripts/pmc_sq2.sh r05j_c2 > $O/sq_c2.log 2>&1 || { tail -5 $O/sq_c2.log; exit 8; }
BENCH_ARGS="--config hopping_double --steps 1 --warmup 1 --no-cpu-baseline --no-extras" KFILT="k_c1v_(merge|scatter|refine)" bash scripts/pmc_sq2.sh r05j_c3 > $O/sq_c3.log 2>&1 || { tail -5 $O/sq_c3.log; exit 8; }
cat $O/sq_c2.log $O/sq_c3.log | cut -c1-220
