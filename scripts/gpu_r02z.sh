#!/bin/bash
# r02z: end-of-round state — every GPU test (fast + full-size parity), smoke, the default bench,
# every bench leg with its CPU baseline, rocprofv3 evidence (kernel stats + FETCH/WRITE traffic)
# for the C2 and C3 legs.  The first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ITAG=${ITAG:-r02z}
D=gpurun_out/$ITAG
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread \
  > $D/gpu_all.log 2>&1; rc=$?
tail -5 $D/gpu_all.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u __graft_entry__.py smoke > $D/smoke.log 2>&1 || { echo smoke failed; cat $D/smoke.log; exit 3; }
timeout -k 10 400 python -u bench.py > $D/bench.jsonl 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 4; }
cut -c1-400 $D/bench.jsonl
for L in hourly_metrics hopping_double clickstream_join repartition_sum serde_json table_agg session; do
  timeout -k 10 400 python -u bench.py --config $L > $D/leg_$L.jsonl 2> $D/leg_$L.err || { echo "leg $L failed"; tail -20 $D/leg_$L.err; exit 5; }
  cut -c1-300 $D/leg_$L.jsonl
done
STEPS=3 bash scripts/profile_leg.sh $ITAG possible_fraud || exit 6
STEPS=2 bash scripts/profile_leg.sh $ITAG hopping_double || exit 7
echo done
