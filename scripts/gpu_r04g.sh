#!/bin/bash
# Round 4: the COUNT(*) pipeline after the merge's LDS-only barriers / two-chunk prefetch /
# descriptor prefetch and the scatter's per-wave ts stats: bench lines, kernel stats, SQ counters
# and HBM traffic of the c1 kernels, then the parity suites touched this round.  A step that ends
# other than passed (0) or failed-tests (1) — a fault, abort or time limit — ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04g
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E "passed|failed|FAILED|Error|^\{" $O/$name.log | cut -c1-240 | tail -8
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/$name.log; exit $rc; fi
}
run c1 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_c1.py
run bench 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
run sparse 200 python3 bench.py --sparse-keys --steps 20 --warmup 3 --no-cpu-baseline --no-extras
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $R/$O/prof.log 2>&1; echo "prof rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/prof/run_kernel_stats.csv > $O/c2_stats.md; grep -E "k_c1|k_part|k_scan" $O/c2_stats.md
RX=k_c1 timeout -k 10 400 bash scripts/pmc_kernel.sh r04g "--steps 3 --warmup 1 --no-cpu-baseline --no-extras" > $O/pmc.log 2>&1; echo "pmc rc=$?"; cat $O/pmc.log | cut -c1-250
run td 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_time_domains.py
run knobs 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_knobs.py
run parity 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_shuffle.py tests/test_gpu_pull.py
