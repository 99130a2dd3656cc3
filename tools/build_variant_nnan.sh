#!/bin/bash
# A/B variant library with -fno-honor-nans on the attention sources (not misc.hip: its grad-norm check needs isfinite)
#   tools/build_variant_nnan.sh <name> "<-D flags>"
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
mkdir -p build/var_$name
objs=""
for f in cesm_emulator_amd/csrc/*.hip; do
  case $(basename "$f") in tblock.hip|tflash.hip|attn.hip) extra="-fno-slp-vectorize -fno-honor-nans";; sla_fused.hip) extra=-fno-honor-nans;; *) extra=;; esac
  o=build/var_$name/$(basename "$f" .hip).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I include $extra $flags -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined $objs -o cesm_emulator_amd/libcesm_hip_$name.so
