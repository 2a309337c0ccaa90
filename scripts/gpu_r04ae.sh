#!/bin/bash
# Round 4: the probes' emitted-row count over 64 counters (one per block residue) instead of one
# word every wave adds to — join tests, then C4 dense / sparse, release vs the previous build
# (libksqldb_hip_old3.so), kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ae
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_join_string.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "join or probe or c4 or clickstream" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
VARIANTS="rel old3" KGREP="k_probe" BENCH_ARGS="--config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ae_c4s 2 || exit 4
VARIANTS="rel old3" KGREP="k_probe" BENCH_ARGS="--config clickstream_join --steps 3 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ae_c4 1 || exit 5
# the merges' segment lookup at the finest block (32 / 64 / 128 records) that covers the item
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c1v.py tests/test_gpu_panes.py tests/test_gpu_push_shuffled.py tests/test_gpu_records.py > $O/tests_m.log 2>&1 || { echo "merge tests failed rc=$?"; tail -40 $O/tests_m.log; exit 6; }
tail -1 $O/tests_m.log
VARIANTS="rel old3" KGREP="k_c1v_merge" BENCH_ARGS="--config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ae_c3 2 || exit 7
VARIANTS="rel old3" KGREP="k_c1_merge" bash scripts/ab_bench.sh r04ae_c2 2 || exit 8
VARIANTS="rel old3" KGREP="k_c1v_merge" BENCH_ARGS="--config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ae_c5 1 || exit 9
