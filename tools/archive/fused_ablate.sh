#!/bin/bash
# kernel times of the level-0 fused temporal-block / SLA kernels with and without the wgrad-input
# emission: tools/fused_ablate.sh <tag>  -> gpurun_out/<tag>_abl.txt
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
for e in 1 0; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_tbe$e -o run -- python3 tools/tblock_micro.py 64 5 $e > /dev/null 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_slae$e -o run -- python3 tools/sla_micro.py 5 $e > /dev/null 2>&1
done
for d in tbe1 tbe0 slae1 slae0; do echo "== $d"; python3 tools/kstats.py gpurun_out/${tag}_$d 5 12; done > gpurun_out/${tag}_abl.txt
rm -rf gpurun_out/${tag}_tbe? gpurun_out/${tag}_slae?
