#!/bin/bash
# Round 4: straight-line merge record loops (unconditional clamped chunk loads) — merge tests, then
# release vs the previous build (ksql_amd/libksqldb_hip_old.so) on C2, C5, C3 under kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c1v.py tests/test_gpu_panes.py tests/test_gpu_push_shuffled.py tests/test_gpu_records.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
VARIANTS="rel old" KGREP="k_c1_merge|k_c1v_merge" bash scripts/ab_bench.sh r04ab_c2 2 || exit 4
VARIANTS="rel old" KGREP="k_c1v_merge" BENCH_ARGS="--config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ab_c5 2 || exit 5
VARIANTS="rel old" KGREP="k_c1v_merge" BENCH_ARGS="--config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ab_c3 1 || exit 6
