#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box).
#   1. --kernel-trace --stats            → per-kernel average durations
#   2. --pmc FETCH_SIZE (own pass)       → HBM read bytes   (gfx950: ×2 for wide streams, see guide)
#   3. --pmc WRITE_SIZE (own pass)       → HBM write bytes
# Output under gpurun_out/prof_<tag>/; copy summaries into profiles/.
set -u
TAG=${1:-r01}
shift || true
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 5; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 6; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 7; }
find $OUT -name '*.csv' | head -20
python3 tools/rocprof_summary.py stats $OUT/trace/run_kernel_stats.csv > $OUT/kernel_stats.md
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv 100000000 $OUT/traffic.json
cat $OUT/kernel_stats.md | head -14
