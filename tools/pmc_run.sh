#!/bin/bash
# two counter passes over a micro benchmark: tools/pmc_run.sh <prefix> <script> [args...]
set -e
pre=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $pmc -d gpurun_out/${pre}$i -o run -- python3 "$@" > gpurun_out/${pre}$i.log 2>&1
done
