#!/bin/bash
# A/B library with ONE source file taken from a git revision: tools/build_rev_variant.sh <name> <rev> <file.hip>
#   -> cesm_emulator_amd/libcesm_hip_<name>.so (the other sources from the working tree)
set -e
cd "$(dirname "$0")/.."
name=$1; rev=$2; file=$3
d=build/rev_$name
rm -rf "$d" && mkdir -p "$d"
cp cesm_emulator_amd/csrc/*.hip cesm_emulator_amd/csrc/*.h "$d"/
git show "$rev:cesm_emulator_amd/csrc/$file" > "$d/$file"
objs=""
for f in "$d"/*.hip; do
  case $(basename "$f") in tblock.hip|tflash.hip|attn.hip) noslp="-fno-slp-vectorize -fno-honor-nans";; sla_fused.hip) noslp=-fno-honor-nans;; *) noslp=;; esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -I include $noslp -c "$f" -o "${f%.hip}.o" &
  objs="$objs ${f%.hip}.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined $objs -o cesm_emulator_amd/libcesm_hip_$name.so
