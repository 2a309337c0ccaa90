#!/bin/bash
# Fast GPU suite (every -m "gpu and not slow" test), new test files first.  usage: gpu_quick2.sh <tag> [first test files...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-q}; shift
D=gpurun_out/$TAG
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u -m pytest "$@" -m gpu -v --maxfail=10 --timeout 120 --timeout-method thread > $D/first.log 2>&1; rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" $D/first.log | tail -40
  [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -q --maxfail=20 --timeout 120 --timeout-method thread > $D/gpu_fast.log 2>&1; rc=$?
tail -15 $D/gpu_fast.log
exit $rc
