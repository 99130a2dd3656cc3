#!/bin/bash
# Temporal-attention core A/B: tools/tf_ab.sh <tag> [variant libs...] -> gpurun_out/<tag>_tf.txt
# tools/tflash_time.py at the F = 120 level shapes and the F = 12 C >= 256 level shape, default lib vs each
# variant, twice; the temporal-attention parity tests first.
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "temporal_attention or tflash or tattn" --timeout 120 --timeout-method thread > gpurun_out/${tag}_tf_pytest.log 2>&1
tail -2 gpurun_out/${tag}_tf_pytest.log
out=gpurun_out/${tag}_tf.txt
: > $out
for rep in 1 2; do
  for shp in "120 192 288 1" "120 96 144 1" "120 48 72 1" "120 24 36 1" "12 48 72 8" "12 24 36 8"; do
    echo "default $shp" >> $out
    timeout -k 10 120 python3 tools/tflash_time.py $shp 5 >> $out 2>&1
    for v in "$@"; do
      echo "$v $shp" >> $out
      CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_$v.so timeout -k 10 120 python3 tools/tflash_time.py $shp 5 >> $out 2>&1
    done
  done
done
cat $out
