#!/bin/bash
# counter passes over the long-window attention core (tools/tflash_time.py): tools/pmc_tflash.sh <tag> [F H W B reps pm]
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
args=${*:-120 96 144 1 2 1}
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_IFETCH SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pmc -d gpurun_out/${tag}_pmc$i -o run -- python3 tools/tflash_time.py $args > gpurun_out/${tag}_pmc$i.log 2>&1 || echo "pass $i ($pmc) failed"
done
python3 tools/pmc.py gpurun_out/${tag}_pmc* --match=tflash > gpurun_out/${tag}_pmc.txt
rm -rf gpurun_out/${tag}_pmc[0-9]*
cat gpurun_out/${tag}_pmc.txt
