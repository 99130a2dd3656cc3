#!/bin/bash
# TA (vector-memory address unit) busy counters over the fused-block micros and the conv micro
set -e
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
P="TA_TA_BUSY GRBM_GUI_ACTIVE"
timeout -k 10 90 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/ta_tb -o run -- python3 tools/tblock_micro.py 64 2 0 > gpurun_out/ta_tb.log 2>&1
timeout -k 10 90 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/ta_sla -o run -- python3 tools/sla_micro.py 2 0 > gpurun_out/ta_sla.log 2>&1
timeout -k 10 90 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/ta_cv1 -o run -- python3 tools/conv_micro.py 3 0 > gpurun_out/ta_cv1.log 2>&1
CESM_CONV3X3_V4=1 timeout -k 10 90 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/ta_cv4 -o run -- python3 tools/conv_micro.py 3 0 > gpurun_out/ta_cv4.log 2>&1
