#!/bin/bash
# Sink encoder: the sink tests, then kernel stats of the release library against variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sink
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_sink.py -x -v --timeout 120 --timeout-method thread > gpurun_out/sink/tests.log 2>&1 || { tail -40 gpurun_out/sink/tests.log; exit 4; }
tail -3 gpurun_out/sink/tests.log
VARIANTS="${VARIANTS:-rel}" KGREP="k_sink|k_sk" BENCH_ARGS="--config sink_json --steps 10 --warmup 3 --no-cpu-baseline --no-extras" bash scripts/ab_bench.sh sink 2
