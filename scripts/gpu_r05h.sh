#!/bin/bash
# Round 5: the dictionary (block-aggregated claim lists) on the VARCHAR C2 leg, and size-classed
# traffic for the legs still carrying round-4 FETCH_SIZE figures.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 500 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_dict.py \
  "tests/test_gpu_fullsize.py" -k "dict or utf8" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -1 $O/tests.log
timeout -k 10 300 python3 bench.py --utf8 --steps 5 --warmup 2 --no-cpu-baseline > $O/utf8.jsonl 2> $O/utf8.err || { tail $O/utf8.err; exit 4; }
cut -c1-300 $O/utf8.jsonl
for L in "possible_fraud --utf8" session table_agg "table_agg --sparse-ids" hourly_metrics serde_json serde_avro sink_json; do
  STEPS=2 bash scripts/profile_leg.sh r05h $L > $O/prof_$(echo $L | tr ' -' '__').log 2>&1 || { echo "prof $L failed"; tail -8 $O/prof_$(echo $L | tr ' -' '__').log; exit 7; }
  echo "prof $L ok"
done
