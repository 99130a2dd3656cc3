#!/bin/bash
# per-shape conv timing (tools/conv_timing.py) of the default plan vs the persistent conv3x3p for every 3x3 conv
# (CESM_CONV3X3_V4=1), twice -> gpurun_out/v4_conv.txt
set -e
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
: > gpurun_out/v4_conv.txt
for rep in 1 2; do
  echo "== default" >> gpurun_out/v4_conv.txt
  timeout -k 10 300 python3 tools/conv_timing.py >> gpurun_out/v4_conv.txt 2>/dev/null
  echo "== v4" >> gpurun_out/v4_conv.txt
  CESM_CONV3X3_V4=1 timeout -k 10 300 python3 tools/conv_timing.py >> gpurun_out/v4_conv.txt 2>/dev/null
done
grep "conv total" gpurun_out/v4_conv.txt
