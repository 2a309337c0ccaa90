#!/bin/bash
# Round 4 end-of-round evidence, part 3: per-leg rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE
# passes (scripts/profile_leg.sh), for the legs named in LEGS ("config[:extra-flag]" ...).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for L in ${LEGS}; do
  CFG=${L%%:*}; X=""
  [ "$CFG" != "$L" ] && X="--${L#*:}"
  echo "== $CFG $X"
  bash scripts/profile_leg.sh r04 $CFG $X || { echo "profile $L failed"; exit 6; }
done
