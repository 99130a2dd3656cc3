#!/bin/bash
# A/B variant library: tools/build_variant.sh <name> "<-D flags>" -> cesm_emulator_amd/libcesm_hip_<name>.so
# (load it with CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_<name>.so)
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
mkdir -p build/var_$name
objs=""
for f in cesm_emulator_amd/csrc/*.hip; do
  case $(basename "$f") in tblock.hip|tflash.hip|attn.hip) noslp="-fno-slp-vectorize -fno-honor-nans";; sla_fused.hip) noslp=-fno-honor-nans;; *) noslp=;; esac
  o=build/var_$name/$(basename "$f" .hip).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I include $noslp $flags -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined $objs -o cesm_emulator_amd/libcesm_hip_$name.so.tmp
mv -f cesm_emulator_amd/libcesm_hip_$name.so.tmp cesm_emulator_amd/libcesm_hip_$name.so
