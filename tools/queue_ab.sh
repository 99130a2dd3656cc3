#!/bin/bash
# conv3x3p dynamic item queue vs static split, with and without the co-running weight-gradient stream
# (CESM_WGRAD_STREAM=1, the proxy for RCCL kernels overlapped with the backward): tools/queue_ab.sh <tag>
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_queue_ab.txt
: > $out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_$name" -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --other-configs "" > "gpurun_out/${tag}_$name.json" 2> "gpurun_out/${tag}_$name.err"
  echo "== $name: $(python3 -c "import json,sys; d=json.loads(open('gpurun_out/${tag}_$name.json').read().strip().split(chr(10))[-1]); print(d['value'], d['ms_per_step'])")" >> $out
  python3 tools/kstats.py "gpurun_out/${tag}_$name" 7 200 | grep -E "conv3x3p|total" >> $out
  rm -rf "gpurun_out/${tag}_$name"
}
run dyn CESM_X=0
run static CESM_CONV_STATIC=1
run dyn_wstream CESM_WGRAD_STREAM=1
run static_wstream CESM_WGRAD_STREAM=1 CESM_CONV_STATIC=1
cat $out
