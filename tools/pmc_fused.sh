#!/bin/bash
# three SQ counter passes over the level-0 fused temporal-block and SLA kernels:
#   tools/pmc_fused.sh <tag>   -> gpurun_out/<tag>_{tb,sla}{1,2,3}/
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
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pmc -d gpurun_out/${tag}_tb$i -o run -- python3 tools/tblock_micro.py 64 2 > gpurun_out/${tag}_tb$i.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $pmc -d gpurun_out/${tag}_sla$i -o run -- python3 tools/sla_micro.py 2 > gpurun_out/${tag}_sla$i.log 2>&1
done
python3 tools/pmc.py gpurun_out/${tag}_tb1 gpurun_out/${tag}_tb2 gpurun_out/${tag}_tb3 --match=tw_ > gpurun_out/${tag}_tb.txt
python3 tools/pmc.py gpurun_out/${tag}_sla1 gpurun_out/${tag}_sla2 gpurun_out/${tag}_sla3 --match=sla > gpurun_out/${tag}_sla.txt
rm -rf gpurun_out/${tag}_tb? gpurun_out/${tag}_sla?
