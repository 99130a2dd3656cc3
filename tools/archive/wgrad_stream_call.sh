#!/bin/bash
# the CESM_WGRAD_STREAM=1 slowdown, measured and traced (tools/wgrad_stream_legs.py,
# tools/wgrad_stream_trace.py).   tools/wgrad_stream_call.sh <tag>
set -e
tag=${1:-r5ws}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_legs.txt
: > $out
for sy in step end; do
  CESM_WGRAD_STREAM=0 timeout -k 10 300 python3 tools/wgrad_stream_legs.py 4 AB $sy >> $out 2>&1
  CESM_WGRAD_STREAM=1 timeout -k 10 300 python3 tools/wgrad_stream_legs.py 4 AB $sy >> $out 2>&1
done
grep "^leg" $out
export CESM_WGRAD_STREAM=1
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/${tag}_tr -o run -- \
  python3 tools/wgrad_stream_legs.py 3 AB ${TRACE_SYNC:-end} > gpurun_out/${tag}_tr.log 2>&1
python3 tools/wgrad_stream_trace.py gpurun_out/${tag}_tr 14 > gpurun_out/${tag}_trace.txt 2>&1
rm -rf gpurun_out/${tag}_tr
head -60 gpurun_out/${tag}_trace.txt
