#!/bin/bash
# Round 5: merge phase probe (C3, C2, C5) and the destroy-releases-buffers test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread "tests/test_gpu_time_domains.py::test_destroy_releases_stream_time_buffers" > $O/leak.log 2>&1; tail -2 $O/leak.log
for A in "--config hopping_double --steps 1 --warmup 1" "--steps 3 --warmup 1" "--config repartition_sum --steps 3 --warmup 1"; do
  KSQL_AMD_LIB_VARIANT=tune KHIP_AGG_PROBE=1 timeout -k 10 300 python3 bench.py $A --no-cpu-baseline --no-extras > $O/probe.jsonl 2> $O/probe.err || { tail -5 $O/probe.err; exit 5; }
  echo "== $A"; grep "merge probe" $O/probe.err | tail -3
done
