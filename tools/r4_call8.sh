#!/bin/bash
# Round-4 call 8: the F = 120 per-GPU leg (more_blocks, 192x288, B = 1) profiled as the main config: kernel totals
# and the per-call durations of the temporal-attention and projection kernels.  tools/r4_call8.sh <tag>
set -e
tag=${1:-r4c8}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace -d "gpurun_out/${tag}_f120" -o run -- \
  python3 bench.py --frames 120 --batch 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --other-configs "" \
  > "gpurun_out/${tag}_f120.json" 2> "gpurun_out/${tag}_f120.err"
python3 tools/kstats.py "gpurun_out/${tag}_f120" 3 45 > "gpurun_out/${tag}_f120_summary.txt"
python3 tools/kcalls.py "gpurun_out/${tag}_f120" tflash 40 > "gpurun_out/${tag}_f120_tflash_calls.txt"
python3 tools/kcalls.py "gpurun_out/${tag}_f120" gemm1x1 60 > "gpurun_out/${tag}_f120_gemm_calls.txt"
rm -rf "gpurun_out/${tag}_f120"
head -30 "gpurun_out/${tag}_f120_summary.txt"
cat "gpurun_out/${tag}_f120_tflash_calls.txt"
