#!/bin/bash
# Round 4: dense probe at 32 rows per thread by default — join tests and C4 full-size parity.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04al
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_join_string.py tests/test_gpu_join_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "join or probe or c4 or clickstream or shard" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --config clickstream_join --steps 3 --warmup 1 > $O/leg_clickstream_join.jsonl 2> $O/leg.err || { echo "leg failed"; tail -10 $O/leg.err; exit 4; }
cut -c1-200 $O/leg_clickstream_join.jsonl
