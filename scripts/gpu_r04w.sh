#!/bin/bash
# Round 4: the pipelines' own sub-pass bits (C5's partitions no longer start with two sub-passes);
# c1 / c1v / knob tests; C5 / C2 / C3 lines; C5 merge phase probe (tuning build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E "passed|failed|FAILED|Error|^\{|merge probe" $O/$name.log | cut -c1-250 | tail -14
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/$name.log; exit $rc; fi
}
run c5 300 python3 bench.py --config repartition_sum --steps 5 --warmup 1 --no-cpu-baseline --no-extras
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/profc5 -o run --output-format csv -- python3 $R/bench.py --config repartition_sum --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $R/$O/profc5.log 2>&1; echo "profc5 rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/profc5/run_kernel_stats.csv > $O/c5_stats.md; grep -E "k_c1|k_shuf|k_part" $O/c5_stats.md
cd $R && KSQL_AMD_LIB_VARIANT=tune KHIP_AGG_PROBE=1 run c5probe 300 python3 bench.py --config repartition_sum --steps 2 --warmup 1 --no-cpu-baseline --no-extras
run c2 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
run c3 300 python3 bench.py --config hopping_double --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run c1 600 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c1v.py tests/test_gpu_knobs.py tests/test_gpu_push_shuffled.py
