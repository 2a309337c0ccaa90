#!/bin/bash
# Round 4: one-destination pack in one pass (k_shuf_pack1); shuffle + push_shuffled tests; C5 line
# and kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04t
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
run shuf 500 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_gpu_push_shuffled.py tests/test_gpu_shuffle.py
run c5 300 python3 bench.py --config repartition_sum --steps 5 --warmup 1 --no-cpu-baseline --no-extras
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/profc5 -o run --output-format csv -- python3 $R/bench.py --config repartition_sum --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $R/$O/profc5.log 2>&1; echo "profc5 rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/profc5/run_kernel_stats.csv > $O/c5_stats.md; grep -E "k_c1|k_shuf|k_part" $O/c5_stats.md
cd $R && run c5full 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k c5
