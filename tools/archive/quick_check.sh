#!/bin/bash
# quick GPU iteration: tools/quick_check.sh <tag> [pytest -k expr]
#   pytest -m gpu (optionally -k filtered) -> bench (no cpu baseline) -> per-shape conv timing
set -e
tag=$1
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
if [ -n "$2" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$2" > "gpurun_out/${tag}_pytest.log" 2>&1
else
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "gpurun_out/${tag}_pytest.log" 2>&1
fi
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err"
timeout -k 10 200 python3 tools/conv_timing.py > "gpurun_out/${tag}_conv.txt" 2>&1
