#!/bin/bash
# Round 4 end-of-round evidence, part 1: the whole GPU test suite (one process), then smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_final
mkdir -p $O
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread --maxfail=20 tests > $O/suite.log 2>&1; rc=$?
tail -5 $O/suite.log
grep -E "^FAILED|^ERROR" $O/suite.log | head -20
[ $rc -gt 1 ] && { echo "suite rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 $O/smoke.log
