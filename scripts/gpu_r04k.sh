#!/bin/bash
# Round 4: c1info read through device-coherent loads (the ts-span decline), merge phase probes on
# the tuning build (C2 / C3 / C5), c1 + c1v tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=gpurun_out/r04k
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
run dbg 120 python3 scripts/dbg/ts_span.py
run c1 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_c1.py
run c1v 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_c1v.py
KSQL_AMD_LIB_VARIANT=tune KHIP_AGG_PROBE=1 run p2 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_AGG_PROBE=1 run p5 300 python3 bench.py --config repartition_sum --steps 2 --warmup 1 --no-cpu-baseline --no-extras
KSQL_AMD_LIB_VARIANT=tune KHIP_AGG_PROBE=1 run p3 300 python3 bench.py --config hopping_double --steps 1 --warmup 1 --no-cpu-baseline --no-extras
grep -h "merge probe" $O/p2.log | tail -2; grep -h "merge probe" $O/p5.log | tail -2; grep -h "merge probe" $O/p3.log | tail -3
run bench 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras
