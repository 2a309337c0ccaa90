#!/bin/bash
# Round 4: the step-run layout (no histogram pass: the scatters write each step as one run, the
# refines read chunks from the runs): c1 / c1v / time-domain / knob / full-size tests, C2 / C3 /
# C5 lines, C2 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04q
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E "passed|failed|FAILED|Error|^\{" $O/$name.log | cut -c1-300 | tail -14
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/$name.log; exit $rc; fi
}
run c1 500 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c1v.py tests/test_gpu_time_domains.py
run c2 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/profc2 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $R/$O/profc2.log 2>&1; echo "profc2 rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/profc2/run_kernel_stats.csv > $O/c2_stats.md; grep -E "k_c1|k_part|ksort" $O/c2_stats.md
cd $R && run c3 300 python3 bench.py --config hopping_double --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run c5 300 python3 bench.py --config repartition_sum --steps 5 --warmup 1 --no-cpu-baseline --no-extras
run c2s 200 python3 bench.py --sparse-keys --steps 10 --warmup 2 --no-cpu-baseline --no-extras
run knobs 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_knobs.py
run full 900 python -u -m pytest -q -x --timeout 500 --timeout-method thread tests/test_gpu_fullsize.py -k "c2 or c3 or c5"
