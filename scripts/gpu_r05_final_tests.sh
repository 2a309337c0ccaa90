#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
ITAG=r05_fa PART=tests bash scripts/gpu_final.sh
