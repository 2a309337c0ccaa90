set -o pipefail
mkdir -p gpurun_out/r8a
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_records.py "tests/test_gpu_fullsize.py::test_c2_possible_fraud_full" tests/test_gpu_parity.py > gpurun_out/r8a/tests.log 2>&1 || { tail -30 gpurun_out/r8a/tests.log; exit 3; }
tail -3 gpurun_out/r8a/tests.log
VARIANTS="base rel" bash scripts/ab_bench.sh r8a 2
