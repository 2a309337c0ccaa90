#!/bin/bash
# A/B of tuning knobs on the tuning build (libksqldb_hip_tune.so, KHIP_* read from the env), each
# setting under rocprofv3 kernel stats, alternating for `rounds` rounds.
#   AB="KHIP_R8=0|KHIP_R8=1" ab_knobs.sh <tag> [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abk_${1:-x}
mkdir -p $OUT
export TMPDIR=/tmp KSQL_AMD_LIB_VARIANT=tune
IFS='|' read -ra SETS <<< "${AB:?AB=\"K=v|K=v\"}"
for r in $(seq 1 ${2:-2}); do
  i=0
  for S in "${SETS[@]}"; do
    i=$((i + 1))
    tag=s${i}r$r
    env $S timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu-baseline --no-extras} > $OUT/$tag.log 2>&1 || { echo "$S failed"; tail -5 $OUT/$tag.log; exit 5; }
    echo "== [$S] r$r: $(python3 -c "import json;d=json.loads([l for l in open('$OUT/$tag.log') if l.startswith('{')][-1]);print('%.3e rec/s step %.3f ms'%(d['value'],d['ms_per_step']))")"
    python3 tools/rocprof_summary.py stats $OUT/$tag/run_kernel_stats.csv | grep -E "${KGREP:-k_part_(merge|scatter|refine|hist)}" | cut -c1-80
  done
done
