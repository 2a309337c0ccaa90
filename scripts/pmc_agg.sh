#!/bin/bash
# Two SQ counter passes over one bench step (instruction mix + wait breakdown); kernel regex $1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
RX=${1:-k_part_agg}
OUT=gpurun_out/sq
mkdir -p $OUT
export TMPDIR=/tmp
BA=${BENCH_ARGS:---steps 1 --warmup 0 --no-cpu-baseline}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $OUT/a -o run --output-format csv -- python3 bench.py $BA > $OUT/a.log 2>&1 || { tail $OUT/a.log; exit 5; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_LDS_ATOMIC_RETURN -d $OUT/b -o run --output-format csv -- python3 bench.py $BA > $OUT/b.log 2>&1 || { tail $OUT/b.log; exit 6; }
for d in a b; do python3 tools/rocprof_summary.py pmc $OUT/$d/run_counter_collection.csv "$RX"; done
