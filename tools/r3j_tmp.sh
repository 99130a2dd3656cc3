#!/bin/bash
set -e
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -k "gn or determinism or repeatable or f120 or F120 or two_stage" --timeout 300 --timeout-method thread > gpurun_out/r3j_pytest.log 2>&1
tail -2 gpurun_out/r3j_pytest.log
tools/f120_round.sh r3j
head -4 gpurun_out/r3j_f120_kernel_summary.txt; grep -E "gn_part|gn_bwd_fin" gpurun_out/r3j_f120_kernel_summary.txt
