#!/bin/bash
# Round 4: straight-line record loop for HOPPING (panes) value merges — value-pipeline tests, then
# C3 release vs the previous build (libksqldb_hip_old4.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ah
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c1v.py tests/test_gpu_panes.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 450 --timeout-method thread tests/test_gpu_fullsize.py -k "c3" > $O/tests_c3.log 2>&1 || { echo "c3 tests failed rc=$?"; tail -40 $O/tests_c3.log; exit 3; }
tail -1 $O/tests_c3.log
VARIANTS="rel old4" KGREP="k_c1v_merge" BENCH_ARGS="--config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ah_c3 2 || exit 4
