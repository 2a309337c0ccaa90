#!/bin/bash
# Hash-probe kernel without its scratch array (k_probe): join parity, then rows-per-thread A/B on
# the sparse-ids C4 leg (tuning build)
set -o pipefail
mkdir -p gpurun_out/probe
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_join_string.py "tests/test_gpu_fullsize.py::test_c4_probe_device_vs_oracle" "tests/test_gpu_fullsize.py::test_c4_clickstream_probe_device_full" tests/test_gpu_parity.py tests/test_gpu_records.py > gpurun_out/probe/tests.log 2>&1 || { tail -30 gpurun_out/probe/tests.log; exit 3; }
tail -2 gpurun_out/probe/tests.log
AB="KHIP_PROBE_PR=4|KHIP_PROBE_PR=8|KHIP_PROBE_PR=16" BENCH_ARGS="--config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras" KGREP="k_probe" bash scripts/ab_knobs.sh pr 1
# grid-strided narrow refine (release) vs one block per workgroup (tuning build): C2 and C1
VARIANTS="tune rel" KGREP="k_part_(refine|scatter|merge)" bash scripts/ab_bench.sh gref 1 || exit 4
VARIANTS="tune rel" BENCH_ARGS="--config hourly_metrics --steps 20 --warmup 3 --no-cpu-baseline --no-extras" KGREP="k_part" bash scripts/ab_bench.sh grefc1 1
