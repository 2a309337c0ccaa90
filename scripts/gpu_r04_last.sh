#!/bin/bash
# Round 4, last check of the final tree: smoke() and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04_last
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_last/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r04_last/smoke.log; exit 3; }
tail -1 gpurun_out/r04_last/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r04_last/bench.jsonl 2> gpurun_out/r04_last/bench.err || { echo "bench failed"; tail -20 gpurun_out/r04_last/bench.err; exit 4; }
cut -c1-240 gpurun_out/r04_last/bench.jsonl
