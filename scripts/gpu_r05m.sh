#!/bin/bash
# Round 5: global (not flat) key-word loads — STRING-key parity, C2 --utf8 both ways, C4 both ways.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05m; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_dict.py tests/test_gpu_join_string.py \
  tests/test_gpu_pull.py tests/test_gpu_serde.py tests/test_gpu_parity.py -k "UTF8 or utf8 or dict or inline or string or pull or serde or join" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
for F in digits alnum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$F -o run --output-format csv -- python3 bench.py --utf8 --card-format $F --steps 10 --warmup 3 --no-cpu-baseline > $O/utf8_$F.jsonl 2> $O/utf8_$F.err || { tail $O/utf8_$F.err; exit 4; }
  grep '^{' $O/utf8_$F.jsonl | cut -c1-200
  python3 tools/rocprof_summary.py stats $O/prof_$F/run_kernel_stats.csv | grep -E "k_dict|k_key|k_c1|fill" | cut -c1-100
done
for X in "" "--sparse-ids"; do
  timeout -k 10 300 python3 bench.py --config clickstream_join $X --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/c4$X.jsonl 2> $O/c4.err || { tail $O/c4.err; exit 5; }
  grep '^{' $O/c4$X.jsonl | cut -c1-200
done
