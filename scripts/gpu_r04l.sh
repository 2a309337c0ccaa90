#!/bin/bash
# Round 4: per-tile late summaries (k_c1_check over tiles, not steps), the join's compact 16-byte
# slots (one INT payload column); c1 / c1v / time-domain / knob / join tests, C2 / C4 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04l
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E "passed|failed|FAILED|Error|^\{|^prod|^oracle|^kt|^\[c1" $O/$name.log | cut -c1-300 | tail -14
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/$name.log; exit $rc; fi
}
run c1 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_c1v.py tests/test_gpu_time_domains.py
run join 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_join_string.py "tests/test_gpu_parity.py::test_qtt_join_golden" "tests/test_gpu_parity.py::test_join_random_vs_oracle" "tests/test_gpu_parity.py::test_join_dense_index_vs_oracle" "tests/test_gpu_fullsize.py::test_c4_probe_device_vs_oracle" "tests/test_gpu_fullsize.py::test_c4_clickstream_probe_device_full"
run bench 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
run c4s 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run c4 300 python3 bench.py --config clickstream_join --steps 3 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_PR=8 run c4s_pr8 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run knobs 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_knobs.py
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $R/$O/prof.log 2>&1; echo "prof rc=$?"
cd $R && python3 tools/rocprof_summary.py stats $O/prof/run_kernel_stats.csv > $O/c2_stats.md; grep -E "k_c1|k_part|k_scan" $O/c2_stats.md
cd $R && run ratomic 150 ./tools/random_atomic && cat $O/ratomic.log
