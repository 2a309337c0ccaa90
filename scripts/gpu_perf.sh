#!/bin/bash
# Parity tests + bench + rocprof (trace, FETCH_SIZE, WRITE_SIZE) in one GPU session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r01}
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider -x > gpurun_out/gpu_tests.log 2>&1; rc=$?; else rc=0; fi
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
BA=${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu-baseline}
timeout -k 10 600 python bench.py $BA > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 4; }
tail -1 gpurun_out/bench.log
for v in ${VARIANTS:-}; do
  env $(echo $v | tr ',' ' ') timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_var.log 2>&1 || { tail -5 gpurun_out/bench_var.log; exit 5; }
  echo "VARIANT $v: $(python3 -c "import json;d=json.loads(open('gpurun_out/bench_var.log').read().strip().splitlines()[-1]);print('%.3e'%d['value'], d['ms_per_step'], d['roofline']['phase_ms_per_step'])")"
done
if [ -n "${PROFILE:-}" ]; then
  bash scripts/profile.sh $TAG || exit 6
  python3 tools/rocprof_summary.py stats gpurun_out/prof_$TAG/trace/run_kernel_stats.csv | head -16
  python3 tools/rocprof_summary.py pmc gpurun_out/prof_$TAG/fetch/run_counter_collection.csv 'k_part|k_apply|k_scan|k_part' 
  python3 tools/rocprof_summary.py pmc gpurun_out/prof_$TAG/write/run_counter_collection.csv 'k_part|k_apply|k_scan'
fi
