#!/bin/bash
# Round 5: block-entry segment lookup (KHIP_C1M_BLK) parity + A/B on C2; single-process pack timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05g; mkdir -p $O
KSQL_AMD_LIB_VARIANT=blk timeout -k 10 400 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_c1.py \
  tests/test_gpu_parity.py tests/test_gpu_time_domains.py > $O/tests_blk.log 2>&1 || { tail -30 $O/tests_blk.log; exit 3; }
tail -1 $O/tests_blk.log
VARIANTS="rel blk" KGREP="k_c1_merge<512, 4, unsigned int" bash scripts/ab_bench.sh r05g_c2 2 || exit 5
timeout -k 10 200 python3 tools/pack_bench.py > $O/pack.jsonl 2> $O/pack.err || { tail $O/pack.err; exit 6; }
cat $O/pack.jsonl
