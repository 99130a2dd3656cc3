#!/bin/bash
# Round-4 call 18: packed 2-wide fp32 VALU ops in the long-window dk / dv kernel and in twh_bwd (libcesm_hip_pk.so,
# -DTF_PK=1 -DTWH_PK=1) -- attention GPU tests with it, then the F = 120 leg and the main leg A/B.  tools/r4_call18.sh <tag>
set -e
tag=${1:-r4c18}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_pk.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v \
  -k "tflash or temporal or decadal or pixel_major" --timeout 400 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1
tail -2 gpurun_out/${tag}_pytest.log
bash tools/env_ab.sh ${tag} --frames 120 --batch 1 --steps 4 --warmup 2 -- - "CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_pk.so"
bash tools/env_ab.sh ${tag}_main --steps 10 --warmup 3 -- - "CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_pk.so"
