#!/bin/bash
# k_part_merge_c1 per-phase wall-clock probe (tuning build, KHIP_AGG_PROBE=1) on the C2 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/probe
export KSQL_AMD_LIB_VARIANT=tune TMPDIR=/tmp
for S in ${SETS:-"KHIP_R8=1"}; do
  env KHIP_AGG_PROBE=1 $S timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/probe/out.log 2> gpurun_out/probe/err.log || { tail -5 gpurun_out/probe/err.log; exit 3; }
  echo "== $S"; grep "probe" gpurun_out/probe/err.log | tail -2
done
