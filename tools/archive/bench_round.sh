#!/bin/bash
# Bench + profile of the current tree: tools/bench_round.sh <tag>
#   1. bench.py (default contract run: headline + other_configs legs + CPU leg) -> gpurun_out/<tag>_bench.json
#   2. rocprofv3 --kernel-trace --stats of the headline step (5 steps)        -> gpurun_out/<tag>_kernel_summary.txt
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 900 python3 bench.py > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --other-configs "" > "gpurun_out/${tag}_prof.json" 2> "gpurun_out/${tag}_prof.err"
python3 tools/kstats.py "gpurun_out/${tag}_prof" 7 60 > "gpurun_out/${tag}_kernel_summary.txt"
rm -rf "gpurun_out/${tag}_prof"
head -30 "gpurun_out/${tag}_kernel_summary.txt"
