#!/bin/bash
# r02e: emission / retention on the GPU (new tests first), then the rest of the fast suite,
# the full-size C2/C3 parity tests and a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${ITAG:-r02e}
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_emit.py tests/test_gpu_parity.py -m gpu -q --maxfail=30 --timeout 120 --timeout-method thread \
  > $D/gpu_emit.log 2>&1; rc=$?
tail -45 $D/gpu_emit.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -q --timeout 120 --timeout-method thread \
  --deselect tests/test_gpu_emit.py --deselect tests/test_gpu_parity.py > $D/gpu_fast.log 2>&1; rc=$?
tail -15 $D/gpu_fast.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -k "c2_possible_fraud_full or c3" -x -v --timeout 600 --timeout-method thread \
  > $D/gpu_full.log 2>&1 || { echo "fullsize tests failed"; tail -40 $D/gpu_full.log; exit 1; }
grep -E "PASSED|FAILED" $D/gpu_full.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $D/bench.jsonl 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 4; }
python3 -c "import json; d=json.loads(open('$D/bench.jsonl').read()); r=d['roofline']; print('value %.3e step %.3f ms frac %.3f' % (d['value'], d['ms_per_step'], r['frac']))"
