#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Every GPU step has its own time
# limit; a crash / timeout ends the script (test assertion failures do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
echo "== host: $(nproc) cpus; $(lscpu | grep 'Model name' | head -1)"
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -q -m gpu -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || { tail -40 gpurun_out/bench.log; exit 4; }
cat gpurun_out/bench.log
