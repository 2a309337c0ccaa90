#!/bin/bash
# Round 4: one-pass pack with 16-byte row stores; probe batch sweep 6 / 8 / 12 (C4 sparse ids);
# shuffle + join tests; C5 / C4 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04v
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
run shuf 500 python -u -m pytest -q -x --timeout 240 --timeout-method thread tests/test_gpu_push_shuffled.py tests/test_gpu_shuffle.py
run c5 300 python3 bench.py --config repartition_sum --steps 5 --warmup 1 --no-cpu-baseline --no-extras
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/profc5 -o run --output-format csv -- python3 $R/bench.py --config repartition_sum --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $R/$O/profc5.log 2>&1; echo "profc5 rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/profc5/run_kernel_stats.csv > $O/c5_stats.md; grep -E "k_c1|k_shuf|k_part" $O/c5_stats.md
cd $R && KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_PR=6 run c4s_pr6 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_PR=8 run c4s_pr8 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_PR=12 run c4s_pr12 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run join 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_join_string.py "tests/test_gpu_parity.py::test_join_random_vs_oracle" "tests/test_gpu_fullsize.py::test_c4_clickstream_probe_device_full"
