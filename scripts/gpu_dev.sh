#!/bin/bash
# Development loop on the GPU box: selected GPU tests, the default bench line, rocprofv3 kernel
# stats of the bench.  usage: ITAG=x TESTS="tests/a.py tests/b.py::t" BENCH_ARGS="..." gpu_dev.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
D=gpurun_out/${ITAG:-dev}
mkdir -p $D
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-500} python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $D/tests.log 2>&1
  rc=$?; tail -4 $D/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $D/tests.log | head -30; exit $rc; }
fi
B=${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline --no-extras}
timeout -k 10 300 python3 bench.py $B > $D/bench.jsonl 2> $D/bench.err || { tail -20 $D/bench.err; exit 4; }
python3 -c "import json;d=json.loads([l for l in open('$D/bench.jsonl') if l.startswith('{')][-1]);print('%s %.4e rec/s step %.3f ms frac %.3f'%(d['config'].get('workload'),d['value'],d['ms_per_step'],d['roofline']['frac']))"
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py $B > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 5; }
  python3 tools/rocprof_summary.py stats $D/prof/run_kernel_stats.csv > $D/kernel_stats.md
  grep -E "k_part|k_scan|k_shuf|k_probe|k_serde|k_sess|k_tagg" $D/kernel_stats.md | head -20 | cut -c1-100
fi
