#!/bin/bash
# Round 4 end-of-round evidence, part 3c: kernel stats + FETCH_SIZE / WRITE_SIZE for the legs the
# value-merge / dictionary changes moved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LEGS="repartition_sum possible_fraud:utf8 possible_fraud" bash scripts/gpu_r04_pmc.sh
