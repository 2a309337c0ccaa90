#!/bin/bash
# Round 4: table aggregation with packed change records and 32-byte source slots (test_tagg, the
# table_agg line + kernel stats); C4 sparse probe batch sweep (PR = 8 / 16).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E "passed|failed|FAILED|Error|^\{" $O/$name.log | cut -c1-400 | tail -14
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/$name.log; exit $rc; fi
}
run tagg 400 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_tagg.py -m gpu
run tagg_bench 300 python3 bench.py --config table_agg --steps 4 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_PR=16 run c4s_pr16 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_PR=8 run c4s_pr8 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --config table_agg --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $R/$O/prof.log 2>&1; echo "prof rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/prof/run_kernel_stats.csv > $O/tagg_stats.md; head -14 $O/tagg_stats.md
