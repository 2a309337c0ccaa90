#!/bin/bash
# Round 4 end-of-round evidence, part 2: the default line and every leg with its CPU baseline
# (bench.py, one process each), then rocprofv3 kernel stats of the default line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_final
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 300 python3 bench.py > $O/leg_default.jsonl 2> $O/leg_default.err || { echo "default failed"; tail -20 $O/leg_default.err; exit 4; }
cut -c1-300 $O/leg_default.jsonl
leg() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/leg_$name.jsonl 2> $O/leg_$name.err || { echo "leg $name failed"; tail -20 $O/leg_$name.err; exit 5; }
  cut -c1-200 $O/leg_$name.jsonl
}
leg possible_fraud_sparse_keys --sparse-keys --steps 10
leg possible_fraud_utf8 --utf8 --steps 5
leg hourly_metrics --config hourly_metrics
leg hopping_double --config hopping_double --steps 3 --warmup 1
leg clickstream_join --config clickstream_join --steps 3 --warmup 1
leg clickstream_join_sparse_ids --config clickstream_join --sparse-ids --steps 3 --warmup 1
leg repartition_sum --config repartition_sum --steps 5 --warmup 1
leg serde_json --config serde_json
leg serde_avro --config serde_avro
leg sink_json --config sink_json
leg table_agg --config table_agg --steps 3 --warmup 1
leg table_agg_sparse_ids --config table_agg --sparse-ids --steps 3 --warmup 1
leg session --config session
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/prof_default.log 2>&1; echo "prof rc=$?"
python3 tools/rocprof_summary.py stats $O/prof_default/run_kernel_stats.csv > $O/kernel_stats_default.md; head -12 $O/kernel_stats_default.md
