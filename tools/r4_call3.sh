#!/bin/bash
# A/B of variant libraries: fused temporal / SLA block kernels (tools/tblock_time.py, every variant twice) and the
# whole bench step (variants named in BENCH_VARIANTS, twice)   tools/r4_call3.sh <tag> <variants...>
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt
: > $out
lib() { if [ "$1" = default ]; then echo cesm_emulator_amd/libcesm_hip.so; else echo cesm_emulator_amd/libcesm_hip_$1.so; fi; }
for rep in 1 2; do
  for v in "$@"; do
    CESM_HIP_LIB=$(lib $v) timeout -k 10 150 python3 tools/tblock_time.py 64 10 >> $out 2>&1
    tail -1 $out
  done
done
for rep in 1 2; do
  for v in ${BENCH_VARIANTS:-$@}; do
    CESM_HIP_LIB=$(lib $v) timeout -k 10 180 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-probe --other-configs "" \
      2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench $v', d['value'], d['ms_per_step'], d.get('loss'))" >> $out
    tail -1 $out
  done
done
