#!/bin/bash
# End-of-round evidence after the R8 / wide kernel changes (ITAG r03y), one GPU call
set -o pipefail
export ITAG=r03y
PART=tests bash scripts/gpu_final.sh || exit $?
LEGS="hopping_double table_agg repartition_sum" PART=legs bash scripts/gpu_final.sh || exit $?
LEGS="hopping_double table_agg repartition_sum" PART=prof bash scripts/gpu_final.sh
