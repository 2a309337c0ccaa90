#!/bin/bash
# Round 4: COUNT(*) pipeline (compact + wide records, cross-item prefetch in the merge) and the
# stream-time domains: tests, C2 full-size parity (dense / sparse / utf8), bench lines, kernel
# stats, merge AU A/B on the tuning build.  A step that ends other than passed (0) or
# failed-tests (1) — a fault, abort or time limit — ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04f
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
run c1 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_c1.py
run td 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_time_domains.py
run bench 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
run sparse 200 python3 bench.py --sparse-keys --steps 20 --warmup 3 --no-cpu-baseline --no-extras
run utf8 200 python3 bench.py --utf8 --steps 20 --warmup 3 --no-cpu-baseline --no-extras
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $R/$O/prof.log 2>&1; echo "prof rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/prof/run_kernel_stats.csv > $O/c2_stats.md; grep -E "k_c1|k_part|k_scan" $O/c2_stats.md
for au in 4 6; do KSQL_AMD_LIB_VARIANT=tune KHIP_C1_AU=$au run au$au 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras; done
run full 800 python -u -m pytest -v --timeout 700 --timeout-method thread tests/test_gpu_fullsize.py -k "c2_possible_fraud"
