#!/bin/bash
# Round 4: the one-destination pack keeping the tile's ts in LDS (read once from HBM) and the key
# dictionary's entry counters spread over 64 words + shrink at 4x — tests, then release vs the
# previous build (libksqldb_hip_old2.so: merge / dictionary changes of r04ac without these).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ad
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shuffle.py tests/test_gpu_push_shuffled.py tests/test_gpu_c1.py tests/test_gpu_join_string.py tests/test_gpu_pull.py tests/test_gpu_emit.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
VARIANTS="rel old2" KGREP="k_shuf_pack1|k_c1v_merge" BENCH_ARGS="--config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ad_c5 2 || exit 4
VARIANTS="rel old2" KGREP="k_dict|k_kid|k_scan_excl|k_c1_merge" BENCH_ARGS="--utf8 --steps 5 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ad_utf8 1 || exit 5
