#!/bin/bash
# Round 4: the straight-line record loop for TUMBLING value merges too (C5's items now hold ~3.8K
# records, 4 chunks) — value-pipeline tests, then C5 release vs the previous build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04aj
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c1v.py tests/test_gpu_push_shuffled.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
VARIANTS="rel old5" KGREP="k_c1v_merge" BENCH_ARGS="--config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04aj_c5 2 || exit 4
