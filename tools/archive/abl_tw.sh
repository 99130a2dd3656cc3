#!/bin/bash
# tw_bwd phase ablations (diagnostic libraries built beforehand by tools/build_variant.sh):
# tools/abl_tw.sh <tag> <variant names...>  -> gpurun_out/<tag>_abl.txt
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_abl.txt
: > $out
timeout -k 10 120 python3 tools/tblock_time.py 64 10 8 >> $out 2>&1
TW_NOEMIT=1 timeout -k 10 120 python3 tools/tblock_time.py 64 10 8 >> $out 2>&1
for v in "$@"; do
  CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so TW_NOEMIT=1 timeout -k 10 120 python3 tools/tblock_time.py 64 10 8 >> $out 2>&1
  CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so timeout -k 10 120 python3 tools/tblock_time.py 64 10 8 >> $out 2>&1
done
