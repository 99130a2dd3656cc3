#!/bin/bash
# Repeatability probe of SLP-vectorized builds (tests/test_gpu_determinism.py, forward + backward of the fused
# temporal block at the level-0 size), one variant library after the other: tools/slp_probe.sh <tag> <variants...>
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/$1_slp_probe.txt; shift
: > $out
for v in "$@"; do
  CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so timeout -k 10 240 python3 -u -m pytest tests/test_gpu_determinism.py \
    -k "temporal_block_repeatable" -x -q --timeout 200 --timeout-method thread > gpurun_out/slp_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep -E 'passed|failed' gpurun_out/slp_$v.log | tail -1) $(grep -m1 'AssertionError' gpurun_out/slp_$v.log)" >> $out
  [ $rc -gt 1 ] && break
done
cat $out
