#!/bin/bash
# Round-4 call 17: query-split dk / dv kernel (tflash_bwd_kv2_kernel, CESM_TF_KV2=1; 4 blocks per CU in the main
# library, 3 in libcesm_hip_kv3.so) -- attention / F = 120 GPU tests with it, then the F = 120 leg A/B.
# tools/r4_call17.sh <tag>
set -e
tag=${1:-r4c17}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
CESM_TF_KV2=1 timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v \
  -k "tflash or temporal_attention or decadal or pixel_major" --timeout 400 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1
tail -2 gpurun_out/${tag}_pytest.log
CESM_TF_KV2=1 CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_kv3.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q \
  -k "temporal_attention_core or pixel_major" --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_kv3.log 2>&1
tail -2 gpurun_out/${tag}_pytest_kv3.log
bash tools/env_ab.sh ${tag} --frames 120 --batch 1 --steps 4 --warmup 2 -- - "CESM_TF_KV2=1" \
  "CESM_TF_KV2=1 CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_kv3.so"
