#!/bin/bash
# Round 5: dictionary rounds without a host round trip between probe and resolve — every STRING-key
# test (forced collisions, growth, joins, table aggregation, pull queries, full size), C1 and C2 --utf8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 900 python -u -m pytest -q -x --timeout 400 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_join_string.py \
  tests/test_tagg.py tests/test_gpu_pull.py tests/test_gpu_emit.py tests/test_gpu_parity.py -k "UTF8 or utf8 or dict or inline or string or pull or tagg or changes" \
  "tests/test_gpu_fullsize.py::test_c2_possible_fraud_utf8_full" "tests/test_gpu_fullsize.py::test_c1_hourly_metrics_full" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/hourly -o run --output-format csv -- python3 bench.py --config hourly_metrics --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $O/hourly.jsonl 2>&1 || exit 4
grep '^{' $O/hourly.jsonl | cut -c1-220
python3 tools/timeline.py $O/hourly/run_kernel_trace.csv k_part_reset | tail -24
for F in digits alnum; do
  timeout -k 10 300 python3 bench.py --utf8 --card-format $F --steps 10 --warmup 3 --no-cpu-baseline > $O/utf8_$F.jsonl 2> $O/utf8_$F.err || { tail $O/utf8_$F.err; exit 5; }
  grep '^{' $O/utf8_$F.jsonl | cut -c1-200
done
