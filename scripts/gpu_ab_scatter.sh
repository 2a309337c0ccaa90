#!/bin/bash
# A/B of the pipelines' scatter against a baseline library (ksql_amd/libksqldb_hip_base.so): the
# release library's c1 / c1v tests, then C2, C5 and C3 under kernel stats, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab_sc
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_c1.py tests/test_gpu_c1v.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_sc/tests.log 2>&1 || { tail -30 gpurun_out/ab_sc/tests.log; exit 4; }
tail -1 gpurun_out/ab_sc/tests.log
VARIANTS="base rel" KGREP="k_c1_(merge|scatter|refine)" BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh sc_c2 2 || exit 5
VARIANTS="base rel" KGREP="k_c1v_(scatter|refine)" BENCH_ARGS="--config repartition_sum --steps 10 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh sc_c5 2 || exit 6
VARIANTS="base rel" KGREP="k_c1v_(scatter|refine)" BENCH_ARGS="--config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh sc_c3 1
