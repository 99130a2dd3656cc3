#!/bin/bash
# A/B timing of variant libraries with tools/tblock_time.py: tools/ab_time.sh <tag> <variants...>
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt
: > $out
for rep in 1 2; do
  timeout -k 10 120 python3 tools/tblock_time.py 64 10 8 >> $out 2>&1
  for v in "$@"; do
    CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so timeout -k 10 120 python3 tools/tblock_time.py 64 10 8 >> $out 2>&1
  done
done
