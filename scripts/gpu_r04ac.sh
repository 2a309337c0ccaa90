#!/bin/bash
# Round 4: (1) key dictionary sized by the key count (retry on probe exhaustion, shrink on reset),
# arena offsets in the probe words, short keys hashed and compared as words; (2) value merge:
# bucket tables read from memory so a 2^12 table of 32-bit identities fits two workgroups per CU,
# barriers of the resident-row phases skipped when a partition has no resident rows.
# Tests, then release vs the previous build (libksqldb_hip_old.so) under kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ac
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c1v.py tests/test_gpu_panes.py tests/test_gpu_push_shuffled.py tests/test_gpu_emit.py tests/test_gpu_join_string.py tests/test_gpu_pull.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 3; }
tail -2 $O/tests.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_serde.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "utf8 or UTF8 or string or varchar or c5 or c3" > $O/tests2.log 2>&1 || { echo "tests2 failed rc=$?"; tail -40 $O/tests2.log; exit 3; }
tail -2 $O/tests2.log
VARIANTS="rel old" KGREP="k_dict|k_kid|k_scan_excl|k_c1_merge" BENCH_ARGS="--utf8 --steps 5 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ac_utf8 1 || exit 4
VARIANTS="rel old" KGREP="k_c1v_merge" BENCH_ARGS="--config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ac_c5 2 || exit 5
VARIANTS="rel old" KGREP="k_c1_merge" bash scripts/ab_bench.sh r04ac_c2 1 || exit 6
VARIANTS="rel old" KGREP="k_c1v_merge" BENCH_ARGS="--config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ac_c3 1 || exit 7
# (3) the one-destination pack keeping the tile's ts in LDS (libksqldb_hip_pk.so) vs release
KSQL_AMD_LIB_VARIANT=pk timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_shuffle.py tests/test_gpu_push_shuffled.py > $O/tests_pk.log 2>&1 || { echo "pk tests failed rc=$?"; tail -30 $O/tests_pk.log; exit 8; }
tail -1 $O/tests_pk.log
VARIANTS="rel pk" KGREP="k_shuf_pack1" BENCH_ARGS="--config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh r04ac_pk 2 || exit 9
