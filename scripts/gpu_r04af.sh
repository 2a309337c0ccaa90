#!/bin/bash
# Round 4: the value pipeline with 64-bit identities (new test) and the value-pipeline suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c1v.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 3; }
grep -E "wide_identity|passed|failed" $O/tests.log | tail -4
