#!/bin/bash
# k_part_merge_c1 phase probe + knob variants (tuning build).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${ITAG:-c1var}
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp KSQL_AMD_LIB_VARIANT=tune
KHIP_AGG_PROBE=1 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $D/probe.log 2>&1 || { tail -20 $D/probe.log; exit 3; }
grep -E "probe" $D/probe.log | tail -2
KHIP_AGG_PROBE=1 KHIP_MERGE_C1=0 timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras > $D/probe0.log 2>&1 || { tail -20 $D/probe0.log; exit 3; }
grep -E "probe" $D/probe0.log | tail -2
VTAG=${ITAG:-c1var}/v bash scripts/gpu_variants2.sh "KHIP_C1_AU=4" "KHIP_C1_AU=8" "KHIP_C1_AU=6"
