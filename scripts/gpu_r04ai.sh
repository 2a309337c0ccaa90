#!/bin/bash
# Round 4: C2 partition count sweep (tuning build, KHIP_PART_LOG2), kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for r in 1 2; do
  for p in 14 15 13; do
    KSQL_AMD_LIB_VARIANT=tune KHIP_PART_LOG2=$p timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/r04ai_${p}_${r}.log 2>&1 || { echo "p=$p failed"; exit 4; }
    echo "p=$p r=$r $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r04ai_${p}_${r}.log') if l.startswith('{')][-1]);print('%.3f ms'%d['ms_per_step'])")"
  done
done
