#!/bin/bash
# Tuning-build knob sweeps on C2 (one GPU call): R8 records per thread per step, COUNT(*) merge chunk
set -o pipefail
AB="KHIP_R8_U=8|KHIP_R8_U=4" bash scripts/ab_knobs.sh r8u 2 || exit 4
AB="KHIP_C1_AU=6|KHIP_C1_AU=8|KHIP_C1_AU=4" bash scripts/ab_knobs.sh c1au 1
