#!/bin/bash
# SQ counter passes over the default bench (one rocprofv3 run per pass, <= 8 SQ counters each),
# summarized for the kernels KFILT matches (default: the partitioned engine's).
#   BENCH_ARGS="--config hopping_double ..." KFILT="k_c1v_merge" pmc_sq2.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/sq_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-extras} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 5; }
  python3 tools/rocprof_summary.py pmc $OUT/p$i/run_counter_collection.csv "${KFILT:-k_part_(merge|scatter|refine|hist)}" >> $OUT/summary.txt
done
cat $OUT/summary.txt
