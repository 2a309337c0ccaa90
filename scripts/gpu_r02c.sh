#!/bin/bash
# r02c: merge-kernel correctness (fast GPU suite + full-size C2/C3) and speed.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/r02c
mkdir -p $D
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 120 --timeout-method thread \
  > $D/gpu_fast.log 2>&1 || { echo "fast gpu tests failed"; tail -40 $D/gpu_fast.log; exit 1; }
tail -2 $D/gpu_fast.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -k "c2_possible_fraud_full or c3" -x -v --timeout 600 --timeout-method thread \
  > $D/gpu_full.log 2>&1 || { echo "fullsize tests failed"; tail -40 $D/gpu_full.log; exit 1; }
grep -E "PASSED|FAILED" $D/gpu_full.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $D/bench_pf.jsonl 2> $D/bench_pf.err \
  || { echo "bench failed"; tail -20 $D/bench_pf.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/bench_pf.jsonl').read()); r=d['roofline']; print('value %.3e step %.3f ms frac %.3f push %.3f ms'%(d['value'], d['ms_per_step'], r['frac'], r['push']['ms']), {k: round(v['ms'],3) for k,v in r['push']['per_kernel'].items()})"
VTAG=r02c/var bash scripts/gpu_variants2.sh X=1 KHIP_MERGE=0
