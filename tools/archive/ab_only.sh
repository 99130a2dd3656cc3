#!/bin/bash
# same-call A/B of the fused attention kernels (tools/tblock_time.py, C = 64 and 128): default lib vs variants
#   tools/ab_only.sh <tag> [variants...]   -> gpurun_out/<tag>_ab.txt
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt
: > $out
for rep in 1 2; do
  for C in 64 128; do
    timeout -k 10 120 python3 tools/tblock_time.py $C 10 8 >> $out 2>&1
    for v in "$@"; do
      CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so timeout -k 10 120 python3 tools/tblock_time.py $C 10 8 >> $out 2>&1
    done
  done
done
grep -v amdgpu.ids $out
