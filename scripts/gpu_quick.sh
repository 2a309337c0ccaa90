#!/bin/bash
# quick: selected GPU tests ($TESTS, pytest args) + a short default bench line
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${ITAG:-quick}
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q --maxfail=20 --timeout 300 --timeout-method thread > $D/tests.log 2>&1; rc=$?
  tail -30 $D/tests.log
  [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > $D/bench.jsonl 2> $D/bench.err || { echo "bench failed"; tail -20 $D/bench.err; exit 4; }
python3 -c "import json; d=json.loads(open('$D/bench.jsonl').read()); r=d['roofline']; print('value %.3e step %.3f ms frac %.3f' % (d['value'], d['ms_per_step'], r['frac']))"
