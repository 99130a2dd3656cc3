#!/bin/bash
# Round-4 call 6: weight-gradient side-stream slowdown by config (host enqueue vs wall, allocator counters), with a
# kernel trace of the slow case.  tools/r4_call6.sh <tag>
set -e
tag=${1:-r4c6}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_stream.txt
: > $out
for cfg in "baseline 8 12" "more_blocks 8 12"; do
  for s in 0 1; do
    CESM_WGRAD_STREAM=$s timeout -k 10 240 python3 -u tools/wgrad_stream_diag.py 5 $cfg >> $out 2>&1
  done
done
cat $out
CESM_WGRAD_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${tag}_tr -o run -- \
  python3 tools/wgrad_stream_diag.py 4 baseline 8 12 > gpurun_out/${tag}_tr.log 2>&1
python3 tools/trace_gaps.py gpurun_out/${tag}_tr 25 > gpurun_out/${tag}_gaps.txt 2>&1 || true
rm -rf gpurun_out/${tag}_tr
head -60 gpurun_out/${tag}_gaps.txt
