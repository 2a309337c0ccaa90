#!/bin/bash
HALF=2 bash "$(dirname "$0")/gpu_r05_final_legs.sh"
