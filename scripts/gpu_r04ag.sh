#!/bin/bash
# Round 4: sharded stream-table join with probe routing, two processes on one GPU over gloo.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04ag
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_join_shard.py > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -60 $O/tests.log; exit 3; }
tail -3 $O/tests.log
