#!/bin/bash
# Round 4 end-of-round evidence after the HOPPING merge loop change: the legs it
# moved, with their CPU baselines (bench.py, one process each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_final4
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
leg() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/leg_$name.jsonl 2> $O/leg_$name.err || { echo "leg $name failed"; tail -20 $O/leg_$name.err; exit 5; }
  cut -c1-200 $O/leg_$name.jsonl
}
timeout -k 10 300 python3 bench.py > $O/leg_default.jsonl 2> $O/leg_default.err || { echo "default failed"; tail -20 $O/leg_default.err; exit 4; }
cut -c1-200 $O/leg_default.jsonl
leg hopping_double --config hopping_double --steps 3 --warmup 1
