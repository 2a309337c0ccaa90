#!/bin/bash
HALF=1 bash "$(dirname "$0")/gpu_r05_final_legs.sh"
