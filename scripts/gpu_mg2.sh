#!/bin/bash
# Generic k_part_merge without register spills (one 512-thread workgroup per CU, KHIP_MG_WPE=2:
# libksqldb_hip_mg2.so) against the release build on C3 and C5; C3 parity first.
set -o pipefail
mkdir -p gpurun_out/mg2
KSQL_AMD_LIB_VARIANT=mg2 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread "tests/test_gpu_fullsize.py::test_c3_bench_push_size" tests/test_gpu_panes.py > gpurun_out/mg2/tests.log 2>&1 || { tail -30 gpurun_out/mg2/tests.log; exit 3; }
tail -2 gpurun_out/mg2/tests.log
VARIANTS="rel mg2" BENCH_ARGS="--config hopping_double --steps 2 --warmup 1 --no-cpu-baseline --no-extras" KGREP="k_part_(merge|scatter|refine)" bash scripts/ab_bench.sh mg2c3 2 || exit 4
VARIANTS="rel mg2" BENCH_ARGS="--config repartition_sum --steps 3 --warmup 1 --no-cpu-baseline --no-extras" KGREP="k_part_(merge|scatter|refine)" bash scripts/ab_bench.sh mg2c5 1
