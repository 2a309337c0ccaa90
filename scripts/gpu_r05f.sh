#!/bin/bash
# Round 5: merge no-load timing experiment (C2), the N=2 pack rehearsal under rocprof, and the
# size-classed traffic passes of the other legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_join_string.py \
  tests/test_gpu_join_shard.py "tests/test_gpu_fullsize.py::test_c4_clickstream_probe_device_full" > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; grep -E "^FAILED" $O/tests.log | head; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python3 bench.py --config clickstream_join --sparse-ids --steps 3 --warmup 1 --no-cpu-baseline > $O/c4s.jsonl 2> $O/c4s.err || exit 4
cut -c1-200 $O/c4s.jsonl
VARIANTS="rel noload" KGREP="k_c1_merge<512, 4, unsigned int" bash scripts/ab_bench.sh r05f_c2 1 || exit 5
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/pack2 -o run_%pid% --output-format csv -- python3 bench.py \
  --config repartition_sum --gpus 2 --exchange gloo --one-device --records 20000000 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-extras > $O/pack2.log 2>&1 || { echo "pack2 failed"; tail -20 $O/pack2.log; exit 6; }
grep '^{' $O/pack2.log | cut -c1-200
for f in $(find $O/pack2 -name "*kernel_stats.csv"); do python3 tools/rocprof_summary.py stats $f | grep -E "k_shuf|k_c1v" | cut -c1-100; done
for L in hopping_double repartition_sum clickstream_join "clickstream_join --sparse-ids" "possible_fraud --sparse-keys"; do
  STEPS=2 bash scripts/profile_leg.sh r05f $L > $O/prof_$(echo $L | tr ' -' '__').log 2>&1 || { echo "prof $L failed"; tail -5 $O/prof_*.log; exit 7; }
  echo "prof $L ok"
done
