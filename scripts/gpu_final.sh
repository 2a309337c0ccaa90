#!/bin/bash
# End-of-round evidence of the committed tree, in parts that each fit one GPU call:
#   PART=tests   every GPU test (fast + full-size parity), smoke, the default bench line, and the
#                C2 leg's rocprofv3 kernel stats + FETCH/WRITE traffic passes
#   PART=legs    every bench leg with its CPU baseline
#   PART=prof    rocprofv3 kernel stats + traffic of the other legs (LEGS to choose)
# The first failure ends the script (tests: a crash or time limit; test failures are reported).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ITAG=${ITAG:-r06_final}
D=gpurun_out/$ITAG
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ALL_LEGS="possible_fraud:--sparse-keys possible_fraud:--utf8 possible_fraud:--utf8:--card-format:alnum hourly_metrics hopping_double clickstream_join clickstream_join:--sparse-ids repartition_sum serde_json serde_avro sink_json table_agg table_agg:--sparse-ids session"
case ${PART:?} in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread \
    > $D/gpu_all.log 2>&1; rc=$?
  tail -5 $D/gpu_all.log
  [ $rc -gt 1 ] && exit $rc
  timeout -k 10 300 python -u __graft_entry__.py smoke > $D/smoke.log 2>&1 || { echo smoke failed; tail $D/smoke.log; exit 3; }
  tail -2 $D/smoke.log
  timeout -k 10 400 python -u bench.py > $D/bench.jsonl 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 4; }
  cut -c1-400 $D/bench.jsonl
  STEPS=3 bash scripts/profile_leg.sh $ITAG possible_fraud || exit 6
  ;;
legs)
  for LA in ${LEGS:-$ALL_LEGS}; do
    L=${LA%%:*}; X=""; [ "$LA" != "$L" ] && X=$(echo "${LA#*:}" | tr ':' ' ')
    T=$L$(echo "$X" | tr -c 'a-z0-9' '_' | sed 's/_*$//')
    timeout -k 10 400 python -u bench.py --config $L $X > $D/leg_$T.jsonl 2> $D/leg_$T.err || { echo "leg $LA failed"; tail -20 $D/leg_$T.err; exit 5; }
    cut -c1-250 $D/leg_$T.jsonl
  done
  ;;
prof)
  for LA in ${LEGS:?}; do
    L=${LA%%:*}; X=""; [ "$LA" != "$L" ] && X=$(echo "${LA#*:}" | tr ':' ' ')
    STEPS=${STEPS:-3} bash scripts/profile_leg.sh $ITAG $L $X > /dev/null || { echo "prof $LA failed"; exit 6; }
    echo "prof $LA ok"
  done
  ;;
esac
echo done
