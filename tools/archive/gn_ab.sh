#!/bin/bash
# GroupNorm chunking A/B: tools/gn_ab.sh <tag> [variant libs...] -> gpurun_out/<tag>_gn.txt
# (tools/gn_time.py at the bench shapes and the F = 120 / B = 1 leg, default lib vs each variant, twice),
# then the GroupNorm parity tests.
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_gn.txt
: > $out
for rep in 1 2; do
  for sh in default f120; do
    GN_SHAPES=$sh timeout -k 10 120 python3 tools/gn_time.py >> $out 2>&1
    for v in "$@"; do
      GN_SHAPES=$sh CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so timeout -k 10 120 python3 tools/gn_time.py >> $out 2>&1
    done
  done
done
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "gn or GN or group" --timeout 120 --timeout-method thread > gpurun_out/${tag}_gn_pytest.log 2>&1
tail -3 gpurun_out/${tag}_gn_pytest.log
cat $out
