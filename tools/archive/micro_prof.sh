#!/bin/bash
# kernel-trace of a micro benchmark: tools/micro_prof.sh <name> <python script> [args...]
set -e
name=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o run -- python3 "$@" > "gpurun_out/$name.log" 2>&1
