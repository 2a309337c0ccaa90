#!/bin/bash
# Round 5: branch-free inline-id pass — STRING-key parity, rows per thread A/B (tuning knob) on C2 --utf8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_join_string.py \
  tests/test_gpu_pull.py tests/test_gpu_parity.py -k "UTF8 or utf8 or dict or inline or string or pull" \
  "tests/test_gpu_fullsize.py::test_c2_possible_fraud_utf8_full" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
BENCH_ARGS="--utf8 --steps 10 --warmup 3 --no-cpu-baseline --no-extras" KGREP="k_key_inline|k_c1_merge<512, 4, unsigned int" \
  AB="KHIP_INLINE_R=1|KHIP_INLINE_R=2|KHIP_INLINE_R=4|KHIP_INLINE_R=8" bash scripts/ab_knobs.sh r05n_utf8 1 || exit 5
