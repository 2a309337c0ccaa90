#!/bin/bash
# Build the library with extra compile flags as ksql_amd/libksqldb_hip_<name>.so (objects in
# ksql_amd/build_<name>/), for an A/B inside one GPU call against the release library
# (scripts/ab_bench.sh: VARIANTS="rel <name>").  Delete variant libraries when the A/B is done.
#   build_variant.sh <name> "<flags>"       e.g. build_variant.sh defer "-DKHIP_C1M_DEFER=1"
set -eu
NAME=$1; FLAGS=${2:-}
cd "$(dirname "$0")/../ksql_amd"
make -s -j8 BUILD=build_$NAME LIB=libksqldb_hip_$NAME.so EXTRA="$FLAGS" libksqldb_hip_$NAME.so
echo "built libksqldb_hip_$NAME.so ($FLAGS)"
