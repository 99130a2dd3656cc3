#!/bin/bash
# whole-step A/B over environment settings: tools/env_ab.sh <tag> <bench args> -- "<ENV=..>" "<ENV=..>" ...
#   "-" stands for the default environment; alternates the settings twice -> gpurun_out/<tag>_env_ab.txt
set -e
tag=$1; shift
args=""
while [ $# -gt 0 ] && [ "$1" != "--" ]; do args="$args $1"; shift; done
[ "$1" == "--" ] && shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_env_ab.txt
: > $out
for rep in 1 2; do
  for v in "$@"; do
    envs=""; [ "$v" != "-" ] && envs="$v"
    env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --other-configs "" $args 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" >> $out
    tail -1 $out
  done
done
cat $out
