#!/bin/bash
# R8 scatter/refine kernels + table-aggregation row-time skip: parity tests, then A/B against the
# previous build (ksql_amd/libksqldb_hip_base.so) on C2 and table_agg.
set -o pipefail
mkdir -p gpurun_out/r8a
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_records.py "tests/test_gpu_fullsize.py::test_c2_possible_fraud_full" tests/test_gpu_parity.py tests/test_tagg.py > gpurun_out/r8a/tests.log 2>&1 || { tail -30 gpurun_out/r8a/tests.log; exit 3; }
tail -3 gpurun_out/r8a/tests.log
VARIANTS="base rel" bash scripts/ab_bench.sh r8a 2 || exit 4
VARIANTS="base rel" BENCH_ARGS="--config table_agg --steps 3 --warmup 1 --no-cpu-baseline --no-extras" KGREP="k_tagg_apply" bash scripts/ab_bench.sh tg1 1
AB="KHIP_REFINE_RECS=8192|KHIP_REFINE_RECS=16384|KHIP_REFINE_RECS=32768" bash scripts/ab_knobs.sh rr 1
