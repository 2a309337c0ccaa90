#!/bin/bash
# Round 4, first call: verify the merged probe/refine change (join + record-layout parity), then
# C2's merge phase breakdown (tuning build, KHIP_AGG_PROBE) and a kernel-stats run of the default
# line, and the sparse-ids probe leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_join_string.py \
  "tests/test_gpu_fullsize.py::test_c4_probe_device_vs_oracle" "tests/test_gpu_fullsize.py::test_c4_clickstream_probe_device_full" \
  tests/test_gpu_parity.py tests/test_gpu_records.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 3; }
tail -2 $O/tests.log
KSQL_AMD_LIB_VARIANT=tune KHIP_AGG_PROBE=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 4; }
grep -E "probe|^\{" $O/probe.log | tail -4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c2 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 5; }
grep '^{' $O/c2.log | cut -c1-200
python3 tools/rocprof_summary.py stats $O/c2/run_kernel_stats.csv | head -24
timeout -k 10 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $O/sparse.log 2>&1 || { tail -20 $O/sparse.log; exit 6; }
grep '^{' $O/sparse.log | cut -c1-300
