#!/bin/bash
# Round 4: c1 ts-span decline diagnostics (tuning build printf), the join's pair-aligned home slots
# (join parity incl. full-size C4 probes, both C4 legs), the random-access ceiling at 64/128 B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04j
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
KSQL_AMD_LIB_VARIANT=tune KHIP_C1_DEBUG=1 run dbg 120 python3 scripts/dbg/ts_span.py
run join 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_join_string.py "tests/test_gpu_parity.py::test_qtt_join_golden" "tests/test_gpu_parity.py::test_join_random_vs_oracle" "tests/test_gpu_parity.py::test_join_dense_index_vs_oracle" "tests/test_gpu_fullsize.py::test_c4_probe_device_vs_oracle" "tests/test_gpu_fullsize.py::test_c4_clickstream_probe_device_full"
run c4s 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras
run c4 300 python3 bench.py --config clickstream_join --steps 3 --warmup 1 --no-cpu-baseline --no-extras
for pr in 1 8; do KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_PR=$pr run c4s_pr$pr 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras; done
timeout -k 10 300 ./tools/random_gather > $O/random_gather.csv 2>&1; echo "rg rc=$?"; cat $O/random_gather.csv
