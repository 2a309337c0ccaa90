#!/bin/bash
# Round 4 end-of-round evidence after the merge / dictionary changes: the GPU suite + smoke
# (scripts/gpu_r04_tests.sh), then the legs those changes moved (C5, C2 --utf8, C3, C2 default)
# with their CPU baselines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r04_tests.sh || exit $?
O=gpurun_out/r04_final
export TMPDIR=/tmp PYTHONUNBUFFERED=1
leg() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/leg_$name.jsonl 2> $O/leg_$name.err || { echo "leg $name failed"; tail -20 $O/leg_$name.err; exit 5; }
  cut -c1-200 $O/leg_$name.jsonl
}
timeout -k 10 300 python3 bench.py > $O/leg_default.jsonl 2> $O/leg_default.err || { echo "default failed"; tail -20 $O/leg_default.err; exit 4; }
cut -c1-200 $O/leg_default.jsonl
leg repartition_sum --config repartition_sum --steps 5 --warmup 1
leg possible_fraud_utf8 --utf8 --steps 5
leg hopping_double --config hopping_double --steps 3 --warmup 1
