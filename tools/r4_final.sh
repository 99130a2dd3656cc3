#!/bin/bash
# Round-4 evidence of the current tree: tools/r4_final.sh <tag>
#   1. PMC HBM traffic passes over one bench step -> profiles/step_traffic.json (bench.py's roofline.traffic)
#   2. pytest -m gpu, smoke()
#   3. bench.py (default contract run)
#   4. rocprofv3 --kernel-trace --stats of the headline step -> kernel summary
#   5. SQ counter passes over one step for the dominant kernels
#   6. the F = 120 leg profiled as the main config (kernel totals, per-call attention / projection durations)
# Each GPU step has its own time limit; the first failure ends the call.
set -e
tag=${1:-r4f}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/libcesm_hip.so > gpurun_out/${tag}_md5.txt
bash tools/pmc_traffic.sh ${tag} > gpurun_out/${tag}_traffic.log 2>&1
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "gpurun_out/${tag}_pytest.log" 2>&1
tail -2 "gpurun_out/${tag}_pytest.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${tag}_smoke.log" 2>&1
tail -2 "gpurun_out/${tag}_smoke.log"
timeout -k 10 600 python3 bench.py > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err"
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'], {k: v.get('ms_per_step') for k, v in d.get('other_configs', {}).items()})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --other-configs "" > "gpurun_out/${tag}_prof.json" 2> "gpurun_out/${tag}_prof.err"
python3 tools/kstats.py "gpurun_out/${tag}_prof" 7 60 > "gpurun_out/${tag}_kernel_summary.txt"
rm -rf "gpurun_out/${tag}_prof"
head -14 "gpurun_out/${tag}_kernel_summary.txt"
PMC_KERNELS="conv3x3_bf16_kernelILi36ELi7 conv3x3ws twh_bwd slah_dx wgrad3x3c64" bash tools/pmc_step_sq.sh ${tag} > gpurun_out/${tag}_sq.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace -d "gpurun_out/${tag}_f120" -o run -- \
  python3 bench.py --frames 120 --batch 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --other-configs "" \
  > "gpurun_out/${tag}_f120.json" 2> "gpurun_out/${tag}_f120.err"
python3 tools/kstats.py "gpurun_out/${tag}_f120" 3 45 > "gpurun_out/${tag}_f120_summary.txt"
python3 tools/kcalls.py "gpurun_out/${tag}_f120" tflash 40 > "gpurun_out/${tag}_f120_tflash_calls.txt"
rm -rf "gpurun_out/${tag}_f120"
head -16 "gpurun_out/${tag}_f120_summary.txt"
