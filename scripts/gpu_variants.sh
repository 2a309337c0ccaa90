#!/bin/bash
# Bench variants (env assignments, comma separated per variant) + per-kernel times of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  env $(echo "$v" | tr ',' ' ') timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/var/$i -o run --output-format csv -- python3 bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > gpurun_out/var/$i.log 2>&1 || { tail -5 gpurun_out/var/$i.log; exit 5; }
  echo "== $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/var/$i.log').read().strip().splitlines()[-1]);print('%.3e rec/s push %.3f ms'%(d['value'],d['roofline'].get('push_ms',0)))")"
  python3 tools/rocprof_summary.py stats gpurun_out/var/$i/run_kernel_stats.csv | grep -E "k_part_(scatter|refine|agg|hist)" | cut -c1-80
done
