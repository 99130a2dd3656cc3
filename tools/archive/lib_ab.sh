#!/bin/bash
# Same-call A/B of variant libraries on the whole bench step (plus tools/gn_time.py once per library):
#   tools/lib_ab.sh <tag> <variants...>   (variant v = cesm_emulator_amd/libcesm_hip_<v>.so; "default" = in-tree)
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_lib_ab.txt
: > $out
lib() { if [ "$1" = default ]; then echo cesm_emulator_amd/libcesm_hip.so; else echo cesm_emulator_amd/libcesm_hip_$1.so; fi; }
for v in "$@"; do
  echo "== gn_time $v" >> $out
  CESM_HIP_LIB=$(lib $v) timeout -k 10 120 python3 tools/gn_time.py >> $out 2>&1
  CESM_HIP_LIB=$(lib $v) timeout -k 10 120 python3 tools/wred_time.py >> $out 2>&1
done
for rep in 1 2; do
  for v in "$@"; do
    echo "== bench $v rep $rep" >> $out
    CESM_HIP_LIB=$(lib $v) timeout -k 10 180 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe \
      2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d.get('loss'))" >> $out
  done
done
cat $out
