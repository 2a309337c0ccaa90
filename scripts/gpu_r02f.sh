#!/bin/bash
# r02f: state check after the second re-entry — every fast GPU test, smoke, default bench, then
# rocprofv3 evidence per bench leg (kernel stats + FETCH/WRITE traffic; SQ counters for C2).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ITAG=${ITAG:-r02f}
D=gpurun_out/$ITAG
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -q --maxfail=20 --timeout 120 --timeout-method thread \
  > $D/gpu_fast.log 2>&1; rc=$?
tail -25 $D/gpu_fast.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $D/smoke.log 2>&1 || { echo smoke failed; cat $D/smoke.log; exit 3; }
timeout -k 10 400 python -u bench.py > $D/bench.jsonl 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 4; }
cat $D/bench.jsonl
[ "${PROF:-1}" = 1 ] || exit 0
SQ=1 STEPS=3 bash scripts/profile_leg.sh $ITAG possible_fraud || exit 5
STEPS=2 bash scripts/profile_leg.sh $ITAG hopping_double || exit 6
STEPS=3 bash scripts/profile_leg.sh $ITAG clickstream_join || exit 7
STEPS=3 bash scripts/profile_leg.sh $ITAG repartition_sum || exit 8
STEPS=3 bash scripts/profile_leg.sh $ITAG hourly_metrics || exit 9
echo done
