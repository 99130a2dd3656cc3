#!/bin/bash
# Validation of the current tree: full GPU suite + contract bench main leg.  tools/r4_check.sh <tag>
set -e
tag=${1:-r4chk}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/libcesm_hip.so > gpurun_out/${tag}_md5.txt
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "gpurun_out/${tag}_pytest.log" 2>&1
tail -2 "gpurun_out/${tag}_pytest.log"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --other-configs "" > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err"
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
