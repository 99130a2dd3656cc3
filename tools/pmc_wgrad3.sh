#!/bin/bash
# SQ counter passes over the 3x3 conv at U-Net level $1 (tools/conv_micro.py): tools/pmc_conv3.sh <level> <tag>
set -e
lvl=$1; tag=$2
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pmc -d gpurun_out/${tag}_$i -o run -- python3 tools/wgrad_micro.py 3 $lvl > gpurun_out/${tag}_$i.log 2>&1
done
python3 tools/pmc.py gpurun_out/${tag}_1 gpurun_out/${tag}_2 gpurun_out/${tag}_3 --match=wgrad > gpurun_out/${tag}.txt
rm -rf gpurun_out/${tag}_?
