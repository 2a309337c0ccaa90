#!/bin/bash
# SQ counter passes (one rocprofv3 run each, at most 8 SQ counters) over a bench command; summary
# for the kernels matching $RX.  usage: pmc_kernel.sh <tag> "<bench args>"
set -u
TAG=$1; ARGS=$2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
RX=${RX:-k_part}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 5; }
  python3 tools/rocprof_summary.py pmc $OUT/p$i/run_counter_collection.csv "$RX" | tee -a $OUT/summary.txt
done
