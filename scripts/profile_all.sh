#!/bin/bash
# rocprofv3 evidence for every bench leg (run on the GPU box).
#   possible_fraud: --kernel-trace --stats, then --pmc FETCH_SIZE and --pmc WRITE_SIZE in their own passes
#   hopping_double, clickstream_join: --kernel-trace --stats
# Output under gpurun_out/prof_<tag>/; copy summaries into profiles/<round>/.
set -u
TAG=${1:-r01c}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="--steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/pf -o run --output-format csv -- python3 bench.py $B > $OUT/pf.log 2>&1 || { tail -20 $OUT/pf.log; exit 5; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 6; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 7; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c3 -o run --output-format csv -- python3 bench.py --config hopping_double --steps 2 --warmup 1 --no-cpu-baseline > $OUT/c3.log 2>&1 || { tail -20 $OUT/c3.log; exit 8; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/c4 -o run --output-format csv -- python3 bench.py --config clickstream_join --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c4.log 2>&1 || { tail -20 $OUT/c4.log; exit 9; }
for leg in pf c3 c4; do
  python3 tools/rocprof_summary.py stats $OUT/$leg/run_kernel_stats.csv > $OUT/kernel_stats_$leg.md
done
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv 100000000 $OUT/traffic.json
head -14 $OUT/kernel_stats_pf.md
