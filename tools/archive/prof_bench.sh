#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run: tools/prof_bench.sh <outdir-name> [bench args...]
set -e
name=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"
