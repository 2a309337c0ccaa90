#!/bin/bash
# Build the library of commit $1 as ksql_amd/libksqldb_hip_<name>.so ($2, default "base"): the
# other side of an ab_bench.sh A/B (VARIANTS="base rel") inside one GPU call, since boxes differ
# by up to ~30 % for the same code.  Delete the variant library when the A/B is done.
set -eu
REV=$1
NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/khip_ref.XXXX)
git -C "$ROOT" worktree add -q --detach "$W" "$REV"
make -s -C "$W/ksql_amd" -j8 >/dev/null
cp "$W/ksql_amd/libksqldb_hip.so" "$ROOT/ksql_amd/libksqldb_hip_$NAME.so"
git -C "$ROOT" worktree remove --force "$W"
echo "built $REV as libksqldb_hip_$NAME.so"
