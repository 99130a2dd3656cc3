#!/bin/bash
# Step throughput with the batch source inside the timed region: resident (inputs already in HBM), device
# (DeviceWindowLoader: HBM-resident fields + cesm_window_gather per step), pinned (PinnedWindowLoader: pinned
# host windows, side-stream H2D overlapped with the step).  tools/data_bench.sh <tag> -> gpurun_out/<tag>_data.txt
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
out=gpurun_out/${tag}_data.txt
: > $out
for d in resident device pinned; do
  timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --data $d > gpurun_out/${tag}_data_$d.json 2> gpurun_out/${tag}_data_$d.err
  python3 -c "import json; d=json.load(open('gpurun_out/${tag}_data_$d.json')); print('$d', d['value'], d['ms_per_step'], d.get('data'))" >> $out
done
cat $out
