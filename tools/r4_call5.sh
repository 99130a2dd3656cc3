#!/bin/bash
# Round-4 call 5: defaults = warp-specialized level-0 conv, per-wave tflash dq kernel, weight-gradient side stream
# off.  Full GPU suite, dq old/new check, contract bench, conv bit check, kernel summary.  tools/r4_call5.sh <tag>
set -e
tag=${1:-r4c5}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > "gpurun_out/${tag}_pytest.log" 2>&1
tail -2 "gpurun_out/${tag}_pytest.log"
timeout -k 10 600 python3 -u tools/tf_qw_check.py > gpurun_out/${tag}_qw_check.txt 2>&1
tail -10 gpurun_out/${tag}_qw_check.txt
timeout -k 10 600 python3 bench.py > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err"
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k: v.get('ms_per_step') for k, v in d.get('other_configs', {}).items()})"
timeout -k 10 300 python3 -u tools/ws_check.py > gpurun_out/${tag}_ws_check.txt 2>&1 || true
tail -9 gpurun_out/${tag}_ws_check.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof" -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --other-configs "" > "gpurun_out/${tag}_prof.json" 2> "gpurun_out/${tag}_prof.err"
python3 tools/kstats.py "gpurun_out/${tag}_prof" 7 60 > "gpurun_out/${tag}_kernel_summary.txt"
rm -rf "gpurun_out/${tag}_prof"
head -14 "gpurun_out/${tag}_kernel_summary.txt"
