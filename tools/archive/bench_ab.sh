#!/bin/bash
# whole-step A/B: tools/bench_ab.sh <tag> <extra bench args> -- <variant libs...>
#   bench.py (no CPU leg, no other legs) default lib vs each variant, alternating, twice -> gpurun_out/<tag>_bench_ab.txt
set -e
tag=$1; shift
args=""
while [ $# -gt 0 ] && [ "$1" != "--" ]; do args="$args $1"; shift; done
[ "$1" == "--" ] && shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_bench_ab.txt
: > $out
for rep in 1 2; do
  for v in default "$@"; do
    if [ "$v" == default ]; then lib=""; else lib=cesm_emulator_amd/libcesm_hip_$v.so; fi
    CESM_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --other-configs "" $args 2>>gpurun_out/${tag}_bench_ab.err | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" >> $out
  done
done
cat $out
