#!/bin/bash
# diagnostic library with phase stamps (-DCESM_TW_STAMPS) -> cesm_emulator_amd/libcesm_hip_diag.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build/diag
objs=""
for f in cesm_emulator_amd/csrc/*.hip; do
  case $(basename "$f") in tblock.hip|tflash.hip|attn.hip) noslp=-fno-slp-vectorize;; *) noslp=;; esac
  o=build/diag/$(basename "$f" .hip).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I include $noslp -DCESM_TW_STAMPS $DIAG_FLAGS -c "$f" -o "$o" &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined $objs -o cesm_emulator_amd/libcesm_hip_diag.so
