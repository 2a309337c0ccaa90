#!/bin/bash
# A/B of a COUNT(*) / value pipeline variant library V (ksql_amd/libksqldb_hip_V.so): its tests
# (TESTS, default the COUNT(*) ones), then bench lines under kernel stats, alternating with the
# release library (BENCH_ARGS, KGREP, ROUNDS).   usage: gpu_ab_c1.sh V
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$1
mkdir -p gpurun_out/ab_c1
KSQL_AMD_LIB_VARIANT=$V timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests/test_gpu_c1.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_c1/tests_$V.log 2>&1 || { tail -30 gpurun_out/ab_c1/tests_$V.log; exit 4; }
tail -1 gpurun_out/ab_c1/tests_$V.log
VARIANTS="rel $V" KGREP="${KGREP:-k_c1_(merge|scatter|refine)}" BENCH_ARGS="${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline --no-extras}" bash scripts/ab_bench.sh c1_$V ${ROUNDS:-3}
