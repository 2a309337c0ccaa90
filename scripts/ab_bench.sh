#!/bin/bash
# A/B: library builds under rocprofv3 kernel stats, alternating.  "rel" = the release library,
# any other name V = ksql_amd/libksqldb_hip_V.so (KSQL_AMD_LIB_VARIANT=V).
#   VARIANTS="rel tune" ab_bench.sh <tag> [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 ${2:-2}); do
  for v in ${VARIANTS:-rel tune}; do
    if [ $v = rel ]; then unset KSQL_AMD_LIB_VARIANT; else export KSQL_AMD_LIB_VARIANT=$v; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$v$r -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline --no-extras} > $OUT/$v$r.log 2>&1 || { echo "$v failed"; tail -5 $OUT/$v$r.log; exit 5; }
    echo "== $v$r: $(python3 -c "import json;d=json.loads([l for l in open('$OUT/$v$r.log') if l.startswith('{')][-1]);print('%.3e rec/s step %.3f ms'%(d['value'],d['ms_per_step']))")"
    python3 tools/rocprof_summary.py stats $OUT/$v$r/run_kernel_stats.csv | grep -E "${KGREP:-k_part_(merge|scatter|refine|hist)}" | cut -c1-80
  done
done
