#!/bin/bash
# End of round 5: the legs whose kernels changed after the legs runs (CPU baselines included), then
# rocprofv3 kernel stats + size-classed traffic of the legs whose kernels changed this round.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ITAG=r05_fl PART=legs LEGS="possible_fraud:--utf8 possible_fraud:--utf8:--card-format:alnum hourly_metrics" bash scripts/gpu_final.sh || exit 5
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread "tests/test_gpu_time_domains.py::test_destroy_releases_stream_time_buffers" > gpurun_out/r05_fl/leak_test.log 2>&1; tail -3 gpurun_out/r05_fl/leak_test.log
ITAG=r05_fp PART=prof STEPS=2 LEGS="possible_fraud:--utf8 possible_fraud:--utf8:--card-format:alnum clickstream_join:--sparse-ids hourly_metrics" bash scripts/gpu_final.sh
