#!/bin/bash
# Variant library with the SLP vectorizer ON for every source (incl. the RoPE sources tblock / tflash / attn that
# the product build compiles with -fno-slp-vectorize): cesm_emulator_amd/libcesm_hip_slp.so, for the repeatability
# investigation (tests/test_gpu_determinism.py with CESM_HIP_LIB=...).  Extra flags: tools/build_slp_variant.sh "<flags>" [name]
set -e
cd "$(dirname "$0")/.."
name=${2:-slp}
mkdir -p build/var_$name
objs=""
for f in cesm_emulator_amd/csrc/*.hip; do
  o=build/var_$name/$(basename "$f" .hip).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I include $1 -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined $objs -o cesm_emulator_amd/libcesm_hip_$name.so
