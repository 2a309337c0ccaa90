#!/bin/bash
# Bench variants of the tuning build (KSQL_AMD_LIB_VARIANT=tune): env assignments, comma separated per
# variant; prints value + the partitioned engine's per-kernel average durations (rocprofv3 stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${VTAG:-var2}
mkdir -p $OUT
export TMPDIR=/tmp KSQL_AMD_LIB_VARIANT=tune
i=0
for v in "$@"; do
  i=$((i+1))
  env $(echo "$v" | tr ',' ' ') timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$i -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline --no-extras} > $OUT/$i.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$i.log; exit 5; }
  echo "== $v: $(python3 -c "import json;d=json.loads([l for l in open('$OUT/$i.log') if l.startswith('{')][-1]);print('%.3e rec/s step %.3f ms'%(d['value'],d['ms_per_step']))")"
  python3 tools/rocprof_summary.py stats $OUT/$i/run_kernel_stats.csv | grep -E "k_part|k_scan" | cut -c1-90
  grep "agg probe" $OUT/$i.log | tail -1
done
