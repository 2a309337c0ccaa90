#!/bin/bash
# §8(f) legs on the GPU box: each leg's bench line (with its CPU baseline) + profile_leg.sh evidence.
# usage: gpu_fleg.sh <tag> [legs...]   → gpurun_out/fleg_<tag>/, gpurun_out/prof_<tag>/
set -u
TAG=$1; shift
LEGS=${*:-serde_json table_agg session}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fleg_$TAG
mkdir -p $OUT
for L in $LEGS; do
  echo "== $L"
  timeout -k 10 400 python3 -u bench.py --config $L --steps 5 --warmup 2 > $OUT/$L.json 2> $OUT/$L.err || { tail -30 $OUT/$L.err; exit 3; }
  cat $OUT/$L.json
  bash scripts/profile_leg.sh $TAG $L || exit 4
done
