#!/bin/bash
# Merge-phase probe (tuning build, KHIP_AGG_PROBE=1) + SQ counters of the C2 push kernels.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${ITAG:-probe}
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
KSQL_AMD_LIB_VARIANT=tune KHIP_AGG_PROBE=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $D/probe.log 2>&1 || { tail -20 $D/probe.log; exit 3; }
grep -E "probe" $D/probe.log | tail -3
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $D/sq -o run --output-format csv -- python3 $B > $D/sq.log 2>&1 || { tail -20 $D/sq.log; exit 8; }
python3 tools/rocprof_summary.py pmc $D/sq/run_counter_collection.csv 'k_' > $D/sq_counters.txt
grep -E "k_part" $D/sq_counters.txt | head -30
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $D/sq2 -o run --output-format csv -- python3 $B > $D/sq2.log 2>&1 || { tail -20 $D/sq2.log; exit 9; }
python3 tools/rocprof_summary.py pmc $D/sq2/run_counter_collection.csv 'k_' > $D/sq2_counters.txt
grep -E "k_part" $D/sq2_counters.txt | head -30
