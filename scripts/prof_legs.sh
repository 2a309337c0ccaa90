#!/bin/bash
# rocprofv3 kernel stats of selected bench legs.  LEGS="session table_agg" ITAG=x prof_legs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
D=gpurun_out/${ITAG:-proflegs}
mkdir -p $D
export TMPDIR=/tmp
for L in ${LEGS:?}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/$L -o run --output-format csv -- python3 bench.py --config $L --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-extras ${LEG_ARGS:-} > $D/$L.log 2>&1 || { echo "$L failed"; tail -5 $D/$L.log; exit 5; }
  python3 tools/rocprof_summary.py stats $D/$L/run_kernel_stats.csv > $D/kernel_stats_$L.md
  echo "== $L"; head -16 $D/kernel_stats_$L.md | cut -c1-110
done
