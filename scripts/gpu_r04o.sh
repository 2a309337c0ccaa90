#!/bin/bash
# Round 4: table aggregation with the dense source layout (+ hash layout, transitions), the
# table_agg line dense / sparse ids + kernel stats; C2 with per-wave histograms vs shared (A/B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04o
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
run tagg 400 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_tagg.py -m gpu
run tagg_bench 300 python3 bench.py --config table_agg --steps 4 --warmup 1 --no-cpu-baseline --no-extras
run tagg_sparse 300 python3 bench.py --config table_agg --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run c2 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_C1_HISTW=0 run c2_hist0 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_C1_HISTW=1 run c2_hist1 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
run c1 300 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_gpu_c1.py
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --config table_agg --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $R/$O/prof.log 2>&1; echo "prof rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/prof/run_kernel_stats.csv > $O/tagg_stats.md; head -16 $O/tagg_stats.md
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/profc2 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $R/$O/profc2.log 2>&1; echo "profc2 rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/profc2/run_kernel_stats.csv > $O/c2_stats.md; grep -E "k_c1|k_part" $O/c2_stats.md
