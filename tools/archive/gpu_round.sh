#!/bin/bash
# Full GPU check of the current tree: tools/gpu_round.sh <tag> [skip-tests]
#   1. pytest -m gpu                                   -> gpurun_out/<tag>_pytest.log
#   2. two PMC passes (FETCH_SIZE, WRITE_SIZE) over the bench step at the bench batch (tools/step_pmc.py)
#      -> per-kernel HBM bytes/launch: profiles/step_traffic.json (read by bench.py) + gpurun_out copy
#   3. bench.py (default contract run)                 -> gpurun_out/<tag>_bench.json
#   4. rocprofv3 --kernel-trace --stats of bench.py    -> gpurun_out/<tag>_prof/ (+ kstats summary)
# Every GPU step has its own time limit; steps are chained so the first failure ends the call.
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "gpurun_out/${tag}_pytest.log" 2>&1
fi
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "gpurun_out/${tag}_pmc1" -o run -- \
  python3 tools/step_pmc.py 1 8 12 more_blocks > "gpurun_out/${tag}_pmc1.log" 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "gpurun_out/${tag}_pmc2" -o run -- \
  python3 tools/step_pmc.py 1 8 12 more_blocks > "gpurun_out/${tag}_pmc2.log" 2>&1
python3 tools/step_traffic.py "gpurun_out/${tag}_pmc1" "gpurun_out/${tag}_pmc2" 8 12 more_blocks 1 > "gpurun_out/${tag}_step_traffic.json"
cp "gpurun_out/${tag}_step_traffic.json" profiles/step_traffic.json
rm -rf "gpurun_out/${tag}_pmc1" "gpurun_out/${tag}_pmc2"
timeout -k 10 600 python3 bench.py > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "gpurun_out/${tag}_prof.json" 2> "gpurun_out/${tag}_prof.err"
python3 tools/kstats.py "gpurun_out/${tag}_prof" 7 60 > "gpurun_out/${tag}_kernel_summary.txt"
