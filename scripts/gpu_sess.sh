#!/bin/bash
# SESSION engine: parity tests (emit suite + QTT) then the session bench leg and its profile.
set -u
TAG=${1:-s}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/$TAG; mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_emit.py tests/test_gpu_parity.py -m gpu -q -k "session or qtt or sessions" --maxfail=5 --timeout 120 --timeout-method thread > $D/tests.log 2>&1; rc=$?
tail -8 $D/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --config session --steps 5 --warmup 2 --no-cpu-baseline > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 3; }
cat $D/bench.json
bash scripts/profile_leg.sh $TAG session
