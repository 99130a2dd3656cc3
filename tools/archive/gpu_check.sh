#!/bin/bash
# GPU check of the current tree plus same-call A/B of the fused attention kernels:
#   tools/gpu_check.sh <tag> [variant libs...]   (variant v = cesm_emulator_amd/libcesm_hip_<v>.so)
#   1. pytest -m gpu                                  -> gpurun_out/<tag>_pytest.log
#   2. tools/tblock_time.py at C = 64 and 128, default lib vs each variant, twice
#                                                     -> gpurun_out/<tag>_ab.txt
# Every GPU step has its own time limit; the first failure ends the call.
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "gpurun_out/${tag}_pytest.log" 2>&1
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
tail -3 "gpurun_out/${tag}_pytest.log"
cat $out
