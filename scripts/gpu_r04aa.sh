#!/bin/bash
# Round 4: value-pipeline merge workgroup shape (tuning build knobs KHIP_C1V_NT / KHIP_C1V_LOG2H /
# KHIP_C1V_WG_PER_CU): value-pipeline tests under the 256-thread merge, then C5 and C3 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04aa
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  grep -E "passed|failed|FAILED|Error|^\{" $O/$name.log | sed -E 's/.*"ms_per_step": ([0-9.]+).*/ms \1/' | cut -c1-250 | tail -14
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 $O/$name.log; exit $rc; fi
}
export KSQL_AMD_LIB_VARIANT=tune
T="tests/test_gpu_c1v.py tests/test_gpu_push_shuffled.py tests/test_gpu_panes.py"
KHIP_C1V_NT=256 KHIP_C1V_LOG2H=11 KHIP_C1V_WG_PER_CU=3 run t256 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread $T
B5="python3 bench.py --config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras"
run c5 300 $B5
KHIP_C1V_NT=256 run c5_256 300 $B5
KHIP_C1V_NT=256 KHIP_C1V_LOG2H=11 KHIP_C1V_WG_PER_CU=3 run c5_256_11_3 300 $B5
KHIP_C1V_NT=256 KHIP_C1V_LOG2H=11 KHIP_C1V_WG_PER_CU=4 run c5_256_11_4 300 $B5
KHIP_C1V_LOG2H=11 run c5_512_11 300 $B5
run c5b 300 $B5
B3="python3 bench.py --config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras"
run c3 300 $B3
KHIP_C1V_NT=256 run c3_256 300 $B3
KHIP_C1V_NT=256 KHIP_C1V_LOG2H=11 KHIP_C1V_WG_PER_CU=3 run c3_256_11_3 300 $B3
