#!/bin/bash
# One GPU call of the development loop: selected GPU tests (FIRST, own log), then the whole GPU
# suite, the default bench line and a rocprofv3 kernel-stats run of it.  Test failures (rc 1) do
# not stop the call; a crash, abort or time limit (rc > 1) ends it.
#   ITAG=tag FIRST="tests/test_x.py" SUITE=1 BENCH=1 PROF=1 LEGS="session table_agg" gpu_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${ITAG:-dev}
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -q --timeout 240 --timeout-method thread"
if [ -n "${FIRST:-}" ]; then
  timeout -k 10 ${FIRST_TIMEOUT:-400} $PYT --maxfail=30 $FIRST > $D/first.log 2>&1; rc=$?
  tail -3 $D/first.log
  [ $rc -gt 1 ] && { echo "first tests rc=$rc"; grep -E "Error|FAILED" $D/first.log | head -20; exit $rc; }
  grep -E "^FAILED|Error" $D/first.log | head -20
fi
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 ${SUITE_TIMEOUT:-700} $PYT --maxfail=30 tests > $D/suite.log 2>&1; rc=$?
  tail -3 $D/suite.log
  [ $rc -gt 1 ] && { echo "suite rc=$rc"; grep -E "Error|FAILED" $D/suite.log | head -20; exit $rc; }
  grep -E "^FAILED" $D/suite.log | head -20
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python3 bench.py ${BENCH_ARGS:-} > $D/bench.jsonl 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 4; }
  cut -c1-600 $D/bench.jsonl
fi
for L in ${LEGS:-}; do
  timeout -k 10 400 python3 bench.py --config $L ${LEG_ARGS:-} > $D/leg_$L.jsonl 2> $D/leg_$L.err || { echo "leg $L failed"; tail -20 $D/leg_$L.err; exit 5; }
  cut -c1-400 $D/leg_$L.jsonl
done
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 6; }
  python3 tools/rocprof_summary.py stats $D/prof/run_kernel_stats.csv > $D/kernel_stats.md
  head -25 $D/kernel_stats.md | cut -c1-120
fi
echo done
