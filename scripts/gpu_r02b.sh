#!/bin/bash
# r02b: GPU parity (fast suite + full-size), then the default bench line and the C1 leg.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r02b
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -k "${SEL:-c4 or c5}" -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r02b/gpu_full.log 2>&1 || { echo "fullsize tests failed"; tail -40 gpurun_out/r02b/gpu_full.log; exit 1; }
tail -15 gpurun_out/r02b/gpu_full.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r02b/bench_pf.jsonl 2> gpurun_out/r02b/bench_pf.err \
  || { echo "bench failed"; tail -20 gpurun_out/r02b/bench_pf.err; exit 1; }
cat gpurun_out/r02b/bench_pf.jsonl
timeout -k 10 300 python -u bench.py --config hourly_metrics --steps 20 --warmup 3 > gpurun_out/r02b/bench_c1.jsonl 2> gpurun_out/r02b/bench_c1.err \
  || { echo "bench c1 failed"; tail -20 gpurun_out/r02b/bench_c1.err; exit 1; }
cat gpurun_out/r02b/bench_c1.jsonl
