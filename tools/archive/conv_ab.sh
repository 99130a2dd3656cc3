#!/bin/bash
# conv A/B over one bench step: tools/conv_ab.sh <tag> [variant libs...] -> gpurun_out/<tag>_conv.txt
# (tools/conv_timing.py per-shape totals, default lib vs each variant), conv parity tests first.
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
[ -z "$SKIP_TESTS" ] && timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "conv or gemm or gn" --timeout 120 --timeout-method thread > gpurun_out/${tag}_conv_pytest.log 2>&1
true
tail -2 gpurun_out/${tag}_conv_pytest.log 2>/dev/null || true
out=gpurun_out/${tag}_conv.txt
: > $out
for rep in 1 2; do
  echo "== default" >> $out
  timeout -k 10 300 python3 tools/conv_timing.py >> $out 2>&1
  for v in "$@"; do
    echo "== $v" >> $out
    CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so timeout -k 10 300 python3 tools/conv_timing.py >> $out 2>&1
  done
done
grep -v amdgpu $out | tail -60
