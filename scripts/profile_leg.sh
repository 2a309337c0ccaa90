#!/bin/bash
# rocprofv3 evidence for one bench leg (run on the GPU box), each pass its own run:
#   1. --kernel-trace --stats                          per-kernel average durations (kernel_stats.md)
#   2. --pmc TCC_EA0_RDREQ_{32B,64B,128B}_sum          read requests by size → read bytes (measured)
#   3. --pmc FETCH_SIZE                                cross-check (gfx950 tallies 128-B requests at 64 B)
#   4. --pmc WRITE_SIZE                                write bytes
#   5. [SQ=1] --pmc SQ_*                               wave occupancy / wait breakdown of every kernel
# usage: profile_leg.sh <tag> <config> [extra bench args]   → gpurun_out/prof_<tag>/<config>[...]/
set -u
TAG=$1; CFG=$2; shift 2
EXTRA="$*"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SUF=$(echo "$EXTRA" | tr -c 'a-z0-9' '_' | tr -s '_' | sed 's/_*$//; s/^_*//')
OUT=gpurun_out/prof_$TAG/$CFG${SUF:+_$SUF}
mkdir -p $OUT
export TMPDIR=/tmp
S=${STEPS:-3}; W=1
B="bench.py --config $CFG --steps $S --warmup $W --no-cpu-baseline --no-extras $EXTRA"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $B > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 5; }
python3 tools/rocprof_summary.py stats $OUT/trace/run_kernel_stats.csv > $OUT/kernel_stats.md
head -14 $OUT/kernel_stats.md
timeout -s KILL 600 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $OUT/rdreq -o run --output-format csv -- python3 $B > $OUT/rdreq.log 2>&1 || { tail -20 $OUT/rdreq.log; exit 6; }
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $B > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 6; }
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $B > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 7; }
N=$(python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/trace.log') if l.startswith('{')][-1]); c=d['config']; print(c.get('records_per_gpu') or c.get('clicks_per_gpu') or c.get('rows_per_gpu'))")
python3 tools/pmc_traffic.py $OUT/rdreq/run_counter_collection.csv $OUT/fetch/run_counter_collection.csv $OUT/write/run_counter_collection.csv $N $((S+W)) $OUT/traffic.json $CFG${SUF:+_$SUF}
if [ "${SQ:-0}" = 1 ]; then
  timeout -s KILL 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $OUT/sq -o run --output-format csv -- python3 $B > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 8; }
  python3 tools/rocprof_summary.py pmc $OUT/sq/run_counter_collection.csv 'k_' > $OUT/sq_counters.txt
fi
