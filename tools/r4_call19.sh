#!/bin/bash
# Round-4 call 19: packed fp32 in the long-window forward and dq kernels (libcesm_hip_pk2.so, -DTF_PK2=1)
# -- attention GPU tests with it, then the F = 120 leg A/B.  tools/r4_call19.sh <tag>
set -e
tag=${1:-r4c19}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_pk2.so timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v \
  -k "tflash or temporal or decadal or pixel_major" --timeout 400 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1
tail -2 gpurun_out/${tag}_pytest.log
bash tools/env_ab.sh ${tag} --frames 120 --batch 1 --steps 4 --warmup 2 -- - "CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_pk2.so"
