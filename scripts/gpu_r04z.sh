#!/bin/bash
# Round 4: one-destination pack with 8192-row tiles (KHIP_PACK1_ITEMS=32, tuning build) vs 4096;
# shuffle tests under both; C5 lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04z
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
T="tests/test_gpu_shuffle.py tests/test_gpu_push_shuffled.py"
run shuf 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread $T
KSQL_AMD_LIB_VARIANT=tune KHIP_PACK1_ITEMS=32 run shuf32 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread $T
B="python3 bench.py --config repartition_sum --steps 5 --warmup 2 --no-cpu-baseline --no-extras"
run c5 300 $B
KSQL_AMD_LIB_VARIANT=tune KHIP_PACK1_ITEMS=16 run c5_16 300 $B
KSQL_AMD_LIB_VARIANT=tune KHIP_PACK1_ITEMS=32 run c5_32 300 $B
run c5b 300 $B
KSQL_AMD_LIB_VARIANT=tune KHIP_PACK1_ITEMS=32 run c5_32b 300 $B
grep -h -o '"phases[^}]*}' $O/c5*.log | head
