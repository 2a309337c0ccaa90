#!/bin/bash
# Round 4: the COUNT(*) pipeline after the cstart alignment fix — its own tests first (one at a
# time, stop at the first failure), then the suites and the default line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python -u -m pytest -x -v --timeout 100 --timeout-method thread "tests/test_gpu_c1.py::test_c1_bench_shape" > $O/c1a.log 2>&1 || { tail -40 $O/c1a.log; exit 3; }
grep -E "PASS|FAIL" $O/c1a.log | tail -3
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_c1.py > $O/c1.log 2>&1 || { tail -40 $O/c1.log; exit 4; }
grep -E "PASS|FAIL" $O/c1.log | tail -12
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_time_domains.py > $O/td.log 2>&1 || { tail -40 $O/td.log; exit 8; }
grep -E "PASS|FAIL" $O/td.log | tail -16
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_records.py tests/test_gpu_emit.py "tests/test_gpu_fullsize.py::test_c2_possible_fraud_full" "tests/test_gpu_fullsize.py::test_c2_possible_fraud_utf8_full" > $O/suite.log 2>&1 || { tail -40 $O/suite.log; exit 5; }
tail -2 $O/suite.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 6; }
grep '^{' $O/c2.log | cut -c1-250
python3 tools/rocprof_summary.py stats $O/c2/run_kernel_stats.csv > $O/c2_stats.md; grep -E "k_c1|k_part" $O/c2_stats.md
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2b.log 2>&1 || { tail -20 $O/c2b.log; exit 7; }
grep '^{' $O/c2b.log | cut -c1-200
