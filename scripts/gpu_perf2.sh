#!/bin/bash
# Perf iteration: fast GPU suite (parity), full-size C2/C3 parity, then the default bench under
# rocprofv3 kernel stats.  usage: gpu_perf2.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-perf}
D=gpurun_out/$TAG
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -q -x --timeout 120 --timeout-method thread > $D/gpu_fast.log 2>&1 || { echo "fast gpu tests failed"; tail -30 $D/gpu_fast.log; exit 1; }
tail -1 $D/gpu_fast.log
if [ "${FULL:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -k "c2_possible_fraud_full or c3" -x -v --timeout 600 --timeout-method thread > $D/gpu_full.log 2>&1 || { echo "fullsize tests failed"; tail -40 $D/gpu_full.log; exit 1; }
  grep -E "PASSED|FAILED" $D/gpu_full.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $D/bench.log 2>&1 || { echo "bench failed"; tail -20 $D/bench.log; exit 4; }
python3 -c "import json; d=json.loads([l for l in open('$D/bench.log') if l.startswith('{')][-1]); print('value %.3e step %.3f ms frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))"
python3 tools/rocprof_summary.py stats $D/prof/run_kernel_stats.csv | grep -E "k_part|k_scan" | head -8
