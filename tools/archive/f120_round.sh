#!/bin/bash
# Long-window (BASELINE config 4, F = 120) measurement: tools/f120_round.sh <tag>
#   bench.py --frames 120 --batch 1 -> gpurun_out/<tag>_f120_bench.json ; rocprofv3 summary of the same
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --frames 120 --batch 1 --steps 3 --warmup 2 --no-cpu-baseline --other-configs '' > "gpurun_out/${tag}_f120_bench.json" 2> "gpurun_out/${tag}_f120_bench.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_f120_prof" -o run -- \
  python3 bench.py --frames 120 --batch 1 --steps 3 --warmup 2 --no-cpu-baseline --other-configs '' > "gpurun_out/${tag}_f120_prof.json" 2> "gpurun_out/${tag}_f120_prof.err"
python3 tools/kstats.py "gpurun_out/${tag}_f120_prof" 5 40 > "gpurun_out/${tag}_f120_kernel_summary.txt"
rm -rf "gpurun_out/${tag}_f120_prof"
