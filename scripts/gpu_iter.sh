#!/bin/bash
# One iteration: fast GPU parity suite, the full-size tests selected by $FULL (pytest -k; empty = skip),
# then tuning-build variants of the bench ($@, see gpu_variants2.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${ITAG:-iter}
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread \
  > $D/gpu_fast.log 2>&1 || { echo "fast gpu tests failed"; tail -40 $D/gpu_fast.log; exit 1; }
tail -1 $D/gpu_fast.log
if [ -n "${FULL:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -k "$FULL" -x -v --timeout 600 --timeout-method thread \
    > $D/gpu_full.log 2>&1 || { echo "fullsize tests failed"; tail -40 $D/gpu_full.log; exit 1; }
  grep -E "PASSED|FAILED" $D/gpu_full.log
fi
[ $# -gt 0 ] && VTAG=${ITAG:-iter}/var bash scripts/gpu_variants2.sh "$@"
exit 0
