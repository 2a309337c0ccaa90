#!/bin/bash
# SQ counters for the partitioned engine's kernels (one pass, 8 SQ slots).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-sq}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/log 2>&1 || { tail -20 $OUT/log; exit 5; }
python3 tools/rocprof_summary.py pmc $OUT/run_counter_collection.csv 'k_part'
