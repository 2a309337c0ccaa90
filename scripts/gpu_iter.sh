#!/bin/bash
# Fast iteration loop on the GPU box: parity tests, then a short bench (optionally with
# the agg phase probe).  Each GPU step has its own time limit; a crash ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?
  tail -15 gpurun_out/gpu_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu-baseline} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 4; }
grep -v "^{" gpurun_out/bench.log | tail -4
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
r = d["roofline"]
print("value %.3e rec/s  ms/step %.3f  push %.3f ms  frac %.3f" % (d["value"], d["ms_per_step"], r.get("push_ms", 0), r["frac"]))
for k, v in r.get("per_kernel", {}).items():
    print("  %-16s %.3f ms" % (k, v["ms"]))
PY
