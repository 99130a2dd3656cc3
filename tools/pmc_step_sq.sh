#!/bin/bash
# SQ counter passes (one rocprofv3 run per pass) over one bench training step at the bench batch
# (tools/step_pmc.py), summarised for the dominant attention backwards and forward:
#   tools/pmc_step_sq.sh <tag>  -> gpurun_out/<tag>_sq_<kernel>.txt
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $pmc -d gpurun_out/${tag}_sq$i -o run -- \
    python3 tools/step_pmc.py 1 8 12 more_blocks > gpurun_out/${tag}_sq$i.log 2>&1
done
for k in ${PMC_KERNELS:-twh_bwd slah_dx tw_fwd conv3x3p gn_bwd_apply}; do
  python3 tools/pmc.py gpurun_out/${tag}_sq1 gpurun_out/${tag}_sq2 gpurun_out/${tag}_sq3 --match=$k > gpurun_out/${tag}_sq_$k.txt
done
rm -rf gpurun_out/${tag}_sq1 gpurun_out/${tag}_sq2 gpurun_out/${tag}_sq3
