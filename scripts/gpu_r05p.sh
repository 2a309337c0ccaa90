#!/bin/bash
# Round 5: HOPPING value records combined per (key, pane) in the refine (tuning build, KHIP_C1V_COMB=1)
# — value-pipeline parity with it on, then the C3 A/B against it off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05p; mkdir -p $O
KSQL_AMD_LIB_VARIANT=tune KHIP_C1V_COMB=1 timeout -k 10 700 python -u -m pytest -q -x --timeout 500 --timeout-method thread \
  tests/test_gpu_c1v.py tests/test_gpu_time_domains.py tests/test_gpu_emit.py tests/test_gpu_parity.py -k "HOPPING or hopping or c1v or time or changes or partition or supplied" \
  "tests/test_gpu_fullsize.py::test_c3_hopping_double_microbatches" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
BENCH_ARGS="--config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras" KGREP="k_c1v" \
  AB="KHIP_C1V_COMB=0|KHIP_C1V_COMB=1" bash scripts/ab_knobs.sh r05p_c3 1 || exit 5
