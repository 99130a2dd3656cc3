#!/bin/bash
# Round-4 call 14: pixel-major qkv with the block-per-pixel dq kernels (default) -- attention / F = 120 GPU tests, then
# the F = 120 leg: default vs frame-major vs the per-wave dq kernel.  tools/r4_call14.sh <tag>
set -e
tag=${1:-r4c14}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/libcesm_hip.so > gpurun_out/${tag}_md5.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -k "tflash or temporal_attention or decadal or pixel_major" \
  --timeout 400 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
tail -2 gpurun_out/${tag}_pytest.log
bash tools/env_ab.sh ${tag} --frames 120 --batch 1 --steps 4 --warmup 2 -- - "CESM_TF_PM=0" "CESM_TF_QW=1"
