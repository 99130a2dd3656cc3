#!/bin/bash
# PMC HBM traffic per kernel launch over one bench step at the bench batch (two separate --pmc passes, as
# MI355X_MICROARCH's HBM/rocprofv3 section prescribes) -> profiles/step_traffic.json (read by bench.py for
# roofline.traffic) + a gpurun_out copy: tools/pmc_traffic.sh <tag>
set -e
tag=$1
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "gpurun_out/${tag}_pmc1" -o run -- \
  python3 tools/step_pmc.py 1 8 12 more_blocks > "gpurun_out/${tag}_pmc1.log" 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "gpurun_out/${tag}_pmc2" -o run -- \
  python3 tools/step_pmc.py 1 8 12 more_blocks > "gpurun_out/${tag}_pmc2.log" 2>&1
python3 tools/step_traffic.py "gpurun_out/${tag}_pmc1" "gpurun_out/${tag}_pmc2" 8 12 more_blocks 1 > "gpurun_out/${tag}_step_traffic.json"
cp "gpurun_out/${tag}_step_traffic.json" profiles/step_traffic.json
rm -rf "gpurun_out/${tag}_pmc1" "gpurun_out/${tag}_pmc2"
head -c 1500 "gpurun_out/${tag}_step_traffic.json"
