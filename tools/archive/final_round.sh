#!/bin/bash
# Round-end evidence of the current tree: tools/final_round.sh <tag>
#   1. pytest -m gpu                                   -> gpurun_out/<tag>_pytest.log
#   2. bench.py (default contract run)                 -> gpurun_out/<tag>_bench.json
#   3. rocprofv3 --kernel-trace --stats, headline step -> gpurun_out/<tag>_kernel_summary.txt
# Each GPU step has its own time limit; the first failure ends the call.
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "gpurun_out/${tag}_pytest.log" 2>&1
tail -2 "gpurun_out/${tag}_pytest.log"
timeout -k 10 600 python3 bench.py > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err"
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --other-configs "" > "gpurun_out/${tag}_prof.json" 2> "gpurun_out/${tag}_prof.err"
python3 tools/kstats.py "gpurun_out/${tag}_prof" 7 60 > "gpurun_out/${tag}_kernel_summary.txt"
rm -rf "gpurun_out/${tag}_prof"
head -12 "gpurun_out/${tag}_kernel_summary.txt"
