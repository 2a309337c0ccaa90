#!/bin/bash
# End of round 5: rocprofv3 kernel stats + size-classed traffic of the legs whose kernels changed.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ITAG=r05_fp PART=prof STEPS=2 LEGS="possible_fraud:--utf8 possible_fraud:--utf8:--card-format:alnum clickstream_join:--sparse-ids hourly_metrics" bash scripts/gpu_final.sh
