#!/bin/bash
# split-count sweep of the weight-gradient launches (per-shape conv timing, one bench step each)
set -e
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for nb in 2048 1024 512; do
  CESM_WGRAD_BLOCKS=$nb timeout -k 10 200 python3 tools/conv_timing.py > gpurun_out/wg_$nb.txt 2>&1
done
