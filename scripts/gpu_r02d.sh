#!/bin/bash
# r02d: state check after re-entry — fast GPU suite, every full-size parity test, smoke,
# default bench (with CPU baseline), rocprofv3 kernel stats of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${ITAG:-r02d}
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread \
  > $D/gpu_fast.log 2>&1 || { echo "fast gpu tests failed"; tail -40 $D/gpu_fast.log; exit 1; }
tail -1 $D/gpu_fast.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread \
  > $D/gpu_full.log 2>&1 || { echo "fullsize tests failed"; tail -40 $D/gpu_full.log; exit 1; }
grep -E "PASSED|FAILED" $D/gpu_full.log
timeout -k 10 300 python -u __graft_entry__.py smoke > $D/smoke.log 2>&1 || { echo smoke failed; cat $D/smoke.log; exit 3; }
timeout -k 10 400 python -u bench.py > $D/bench.jsonl 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 4; }
cat $D/bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $D/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $D/prof.log; exit 5; }
python3 tools/rocprof_summary.py stats $D/prof/run_kernel_stats.csv | head -20
