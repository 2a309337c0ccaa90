#!/bin/bash
HALF=2 bash "$(dirname "$0")/gpu_r05_final_legs.sh"
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r05_fl
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_fl/hourly_trace -o run --output-format csv -- python3 bench.py --config hourly_metrics --steps 5 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/r05_fl/hourly_trace.log 2>&1 || exit 9
python3 tools/timeline.py gpurun_out/r05_fl/hourly_trace/run_kernel_trace.csv k_part_reset | tail -40
