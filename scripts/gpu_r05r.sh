#!/bin/bash
# Round 5: COUNT merge with branch-free plane atomics (variant build) — parity, then A/B on C2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05r; mkdir -p $O
KSQL_AMD_LIB_VARIANT=nobr timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_c1.py \
  tests/test_gpu_parity.py -k "c1 or TUMBLING or possible" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
VARIANTS="rel nobr" KGREP="k_c1_merge<512, 4, unsigned int" bash scripts/ab_bench.sh r05r_c2 3 || exit 5
