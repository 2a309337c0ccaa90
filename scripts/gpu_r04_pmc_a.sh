#!/bin/bash
# Round 4 end-of-round evidence, part 3a: kernel stats + FETCH_SIZE / WRITE_SIZE for the legs
# below (scripts/profile_leg.sh), then the SQ_* occupancy / wait pass of C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LEGS="possible_fraud hopping_double repartition_sum table_agg clickstream_join clickstream_join:sparse-ids" bash scripts/gpu_r04_pmc.sh || exit $?
SQ=1 STEPS=2 bash scripts/profile_leg.sh r04sq repartition_sum || exit $?
