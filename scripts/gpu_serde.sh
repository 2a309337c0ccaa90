#!/bin/bash
# serde: parity tests, then both bench legs and their profiles.
set -u
TAG=${1:-t}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/$TAG; mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_serde.py -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -8 $D/tests.log; [ $rc -ne 0 ] && exit $rc
for L in serde_json; do
  timeout -k 10 300 python3 -u bench.py --config $L --steps 5 --warmup 2 --no-cpu-baseline > $D/$L.json 2> $D/$L.err || { tail -20 $D/$L.err; exit 3; }
  cut -c1-300 $D/$L.json
  bash scripts/profile_leg.sh $TAG $L || exit 4
done
