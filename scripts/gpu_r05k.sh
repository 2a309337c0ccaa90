#!/bin/bash
# Round 5: the inline-id pass before the dictionary — STRING-key parity, C2 --utf8 both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -x --timeout 600 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_parity.py \
  tests/test_gpu_join_string.py tests/test_gpu_emit.py tests/test_gpu_pull.py tests/test_gpu_time_domains.py \
  "tests/test_gpu_fullsize.py::test_c2_possible_fraud_utf8_full" "tests/test_gpu_fullsize.py::test_c1_hourly_metrics_full" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for F in digits alnum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$F -o run --output-format csv -- python3 bench.py --utf8 --card-format $F --steps 10 --warmup 3 --no-cpu-baseline > $O/utf8_$F.jsonl 2> $O/utf8_$F.err || { tail $O/utf8_$F.err; exit 4; }
  grep '^{' $O/utf8_$F.jsonl | cut -c1-260
  python3 tools/rocprof_summary.py stats $O/prof_$F/run_kernel_stats.csv | grep -E "k_dict|k_key|k_c1|fill" | cut -c1-100
done
