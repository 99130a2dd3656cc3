#!/bin/bash
# 1x1-conv GEMM A/B: tools/g1_ab.sh <tag> [variant libs...] -> gpurun_out/<tag>_g1.txt (tools/gemm_time.py at the
# F = 12 bench shapes and the F = 120 leg's, default lib vs each variant), conv parity tests first.
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "conv or gemm" --timeout 120 --timeout-method thread > gpurun_out/${tag}_g1_pytest.log 2>&1
tail -2 gpurun_out/${tag}_g1_pytest.log
out=gpurun_out/${tag}_g1.txt
: > $out
for sh in f120 f12; do
  echo "== default $sh" >> $out
  G1_SHAPES=$sh timeout -k 10 200 python3 tools/gemm_time.py >> $out 2>&1
  for v in "$@"; do
    echo "== $v $sh" >> $out
    G1_SHAPES=$sh CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so timeout -k 10 200 python3 tools/gemm_time.py >> $out 2>&1
  done
done
grep -v amdgpu $out
