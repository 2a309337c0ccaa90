#!/bin/bash
# Round 5: hashed-index probe chasing every pending row per round — join parity, C4 --sparse-ids at
# 16 and 8 rows per thread (tuning build knob) against the release build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c1v.py -k "join or c1v or hopping or c3 or c5" \
  tests/test_gpu_join_string.py tests/test_gpu_join_shard.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
BENCH_ARGS="--config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras" KGREP="k_probe" \
  AB="KHIP_PROBE_HPR=16|KHIP_PROBE_HPR=8|KHIP_PROBE_HPR=4" bash scripts/ab_knobs.sh r05l_c4s 1 || exit 5
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_parity.py -k "UTF8 or utf8 or dict or inline" \
  "tests/test_gpu_fullsize.py::test_c2_possible_fraud_utf8_full" > $O/tests_utf8.log 2>&1 || { tail -40 $O/tests_utf8.log; exit 6; }
tail -1 $O/tests_utf8.log
for F in digits alnum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$F -o run --output-format csv -- python3 bench.py --utf8 --card-format $F --steps 10 --warmup 3 --no-cpu-baseline > $O/utf8_$F.jsonl 2> $O/utf8_$F.err || { tail $O/utf8_$F.err; exit 4; }
  grep '^{' $O/utf8_$F.jsonl | cut -c1-200
  python3 tools/rocprof_summary.py stats $O/prof_$F/run_kernel_stats.csv | grep -E "k_dict|k_key|k_c1|fill" | cut -c1-100
done
