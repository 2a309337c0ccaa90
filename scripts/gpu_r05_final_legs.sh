#!/bin/bash
# End of round 5: every bench leg with its CPU baseline (PART=legs of gpu_final.sh), in two calls.
#   HALF=1|2 gpu_r05_final_legs.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
if [ "${HALF:-1}" = 1 ]; then
  LEGS="possible_fraud:--sparse-keys possible_fraud:--utf8 possible_fraud:--utf8:--card-format:alnum hourly_metrics hopping_double clickstream_join clickstream_join:--sparse-ids"
else
  LEGS="repartition_sum serde_json serde_avro sink_json table_agg table_agg:--sparse-ids session"
fi
ITAG=r05_fl PART=legs LEGS="$LEGS" bash scripts/gpu_final.sh
