#!/bin/bash
# LDS pattern probe on the GPU: timings + SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE per pattern kernel
set -e
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 60 tools/lds_probe > gpurun_out/lds_probe.txt 2>&1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/lds_probe_pmc -o run -- tools/lds_probe > /dev/null 2>&1
cat gpurun_out/lds_probe.txt
