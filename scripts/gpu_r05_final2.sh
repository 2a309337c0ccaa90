#!/bin/bash
# Round 5, second end-of-round pass (after the sink, scatter and record-load changes):
#   PART=tests ITAG=r05_fc gpu_final.sh                       (suite, smoke, default line, C2 counters)
#   HALF=1|2 gpu_r05_final2.sh legs                           every leg with its CPU baselines
#   gpu_r05_final2.sh prof                                    kernel stats + counters of the changed legs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
case ${1:?legs|prof} in
legs)
  if [ "${HALF:-1}" = 1 ]; then
    LEGS="possible_fraud:--sparse-keys possible_fraud:--utf8 possible_fraud:--utf8:--card-format:alnum hourly_metrics hopping_double clickstream_join clickstream_join:--sparse-ids"
  else
    LEGS="repartition_sum serde_json serde_avro sink_json table_agg table_agg:--sparse-ids session"
  fi
  ITAG=r05_fl2 PART=legs LEGS="$LEGS" bash scripts/gpu_final.sh ;;
prof)
  ITAG=r05_fp2 PART=prof LEGS="${LEGS:-sink_json hopping_double repartition_sum possible_fraud:--utf8 possible_fraud:--sparse-keys}" bash scripts/gpu_final.sh ;;
esac
