#!/bin/bash
# Wide (32-byte record) scatter/refine kernels: C3/C5/panes parity on the release build, then
# knob A/Bs on the tuning build: KHIP_WK (C3), KHIP_R8_U and KHIP_C1_AU (C2).
set -o pipefail
mkdir -p gpurun_out/wide
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_fullsize.py::test_c3_bench_push_size" "tests/test_gpu_fullsize.py::test_c3_hopping_double_microbatches" "tests/test_gpu_fullsize.py::test_c5_repartition_2p24" tests/test_gpu_panes.py tests/test_gpu_parity.py > gpurun_out/wide/tests.log 2>&1 || { tail -30 gpurun_out/wide/tests.log; exit 3; }
tail -2 gpurun_out/wide/tests.log
AB="KHIP_WK=0|KHIP_WK=1" BENCH_ARGS="--config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras" KGREP="k_part_(merge|scatter|refine)" bash scripts/ab_knobs.sh wk 2 || exit 4
AB="KHIP_R8_U=8|KHIP_R8_U=4" bash scripts/ab_knobs.sh r8u 1 || exit 4
AB="KHIP_C1_AU=6|KHIP_C1_AU=8" bash scripts/ab_knobs.sh c1au 1
