#!/bin/bash
# Round 4 end-of-round evidence, part 3b: kernel stats + FETCH_SIZE / WRITE_SIZE for the legs below.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LEGS="possible_fraud:sparse-keys possible_fraud:utf8 table_agg:sparse-ids session hourly_metrics" bash scripts/gpu_r04_pmc.sh
