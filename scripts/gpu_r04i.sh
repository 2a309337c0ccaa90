#!/bin/bash
# Round 4: ts-range decline fix (LDS flag), value merge specialised by plane shape with word-wise
# row emit; c1 / c1v / knob tests, C2 / C3 / C5 lines and kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04i
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E "passed|failed|FAILED|Error|^\{|^prod|^oracle|^kt" $O/$name.log | cut -c1-300 | tail -12
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/$name.log; exit $rc; fi
}


run c1 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_c1.py
run knobs 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_knobs.py
run c1v 600 python -u -m pytest -v -x --timeout 240 --timeout-method thread tests/test_gpu_c1v.py
run bench 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
run c3 300 python3 bench.py --config hopping_double --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run c5 300 python3 bench.py --config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras


cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $R/$O/prof.log 2>&1; echo "prof rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/prof/run_kernel_stats.csv > $O/c2_stats.md; grep -E "k_c1|k_part|k_scan" $O/c2_stats.md
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof5 -o run --output-format csv -- python3 $R/bench.py --config repartition_sum --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $R/$O/prof5.log 2>&1; echo "prof5 rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/prof5/run_kernel_stats.csv > $O/c5_stats.md; head -16 $O/c5_stats.md
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof3 -o run --output-format csv -- python3 $R/bench.py --config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras > $R/$O/prof3.log 2>&1; echo "prof3 rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/prof3/run_kernel_stats.csv > $O/c3_stats.md; head -16 $O/c3_stats.md

