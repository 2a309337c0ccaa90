#!/bin/bash
# Round 4: grid-strided probe (a few workgroups per CU) vs one workgroup per batch; join tests;
# C4 lines + kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04y
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E "passed|failed|FAILED|Error|^\{" $O/$name.log | cut -c1-250 | tail -14
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/$name.log; exit $rc; fi
}
run join 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_join_string.py "tests/test_gpu_parity.py::test_qtt_join_golden" "tests/test_gpu_parity.py::test_join_random_vs_oracle" "tests/test_gpu_fullsize.py::test_c4_clickstream_probe_device_full"
run c4s 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_GRID=0 run c4s_g0 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_GRID=1024 run c4s_g1k 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_GRID=8192 run c4s_g8k 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/profc4 -o run --output-format csv -- python3 $R/bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $R/$O/profc4.log 2>&1; echo "profc4 rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/profc4/run_kernel_stats.csv > $O/c4_stats.md; head -8 $O/c4_stats.md
