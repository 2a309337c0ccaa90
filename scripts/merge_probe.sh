#!/bin/bash
# Where a leg's merge kernel spends its time: the tuning build's per-phase wall-clock probe
# (KHIP_AGG_PROBE=1: start+evict / records / fold / mark+count+reserve / write, per workgroup) and
# two SQ counter passes (occupancy, waits, LDS instructions and bank conflicts) for kernels matching
# $RX.   usage: merge_probe.sh <tag> "<bench args>"
set -u
TAG=$1; ARGS=$2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mp_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
KSQL_AMD_LIB_VARIANT=tune KHIP_AGG_PROBE=1 timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --no-extras \
  > $OUT/probe.jsonl 2> $OUT/probe.err || { echo "probe run failed"; tail -5 $OUT/probe.err; exit 5; }
grep "merge probe" $OUT/probe.err | tail -4
RX=${RX:-merge} bash scripts/pmc_kernel.sh $TAG "$ARGS --no-cpu-baseline --no-extras" > /dev/null || exit 6
cat gpurun_out/pmc_$TAG/summary.txt
