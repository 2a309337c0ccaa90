#!/bin/bash
# Round 4: dense-index probe rows per thread (tuning build, KHIP_PROBE_DPR 16 / 32 / 64), C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  for d in 16 32 64; do
    KSQL_AMD_LIB_VARIANT=tune KHIP_PROBE_DPR=$d timeout -k 10 300 python3 bench.py --config clickstream_join --steps 3 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/r04ak_${d}_${r}.log 2>&1 || { echo "dpr=$d failed"; tail -5 gpurun_out/r04ak_${d}_${r}.log; exit 4; }
    echo "dpr=$d r=$r $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r04ak_${d}_${r}.log') if l.startswith('{')][-1]);print('%.3f ms %.3e'%(d['ms_per_step'],d['value']))")"
  done
done
