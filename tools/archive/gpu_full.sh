#!/bin/bash
# full GPU test suite of the current tree: tools/gpu_full.sh <tag> -> gpurun_out/<tag>_pytest.log
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "gpurun_out/${tag}_pytest.log" 2>&1
tail -5 "gpurun_out/${tag}_pytest.log"
