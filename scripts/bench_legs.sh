#!/bin/bash
# Every bench.py leg at N=1 (C2 default, C3, C4, C5), one JSON line each under gpurun_out/legs/,
# plus a rocprofv3 kernel-trace summary of the C5 leg.  Each GPU step has its own time limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/legs
for cfg in possible_fraud hopping_double clickstream_join repartition_sum; do
  echo "== $cfg"
  timeout -k 10 400 python bench.py --config $cfg --steps 3 --warmup 1 > gpurun_out/legs/$cfg.log 2>&1 \
    || { tail -30 gpurun_out/legs/$cfg.log; exit 1; }
  grep '^{' gpurun_out/legs/$cfg.log > gpurun_out/legs/$cfg.jsonl
  cut -c1-600 gpurun_out/legs/$cfg.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/legs/prof_c5 -o c5 --output-format csv -- \
  python3 bench.py --config repartition_sum --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/legs/prof_c5.log 2>&1 \
  || { tail -30 gpurun_out/legs/prof_c5.log; exit 2; }
find gpurun_out/legs/prof_c5 -name '*kernel_stats.csv' | head -3
