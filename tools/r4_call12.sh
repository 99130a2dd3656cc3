#!/bin/bash
# Round-4 call 12: pixel-major qkv for the long-window attention (default) vs frame-major (CESM_TF_PM=0): attention and
# F = 120 GPU tests, then the F = 120 leg timed both ways (alternating, twice) with per-call attention durations.
set -e
tag=${1:-r4c12}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -k "tflash or temporal_attention or decadal or pixel_major or ln" \
  --timeout 400 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
tail -3 gpurun_out/${tag}_pytest.log
out=gpurun_out/${tag}_f120_ab.txt
: > $out
for rep in 1 2; do
  for v in 1 0; do
    CESM_TF_PM=$v timeout -k 10 300 python3 bench.py --frames 120 --batch 1 --steps 4 --warmup 2 --no-cpu-baseline \
      --other-configs "" > gpurun_out/${tag}_b.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/${tag}_b.json')); print('PM=$v', d['value'], d['ms_per_step'], [(t['kernel'], t['ms_per_step'], t['avg_us']) for t in d['top_kernels'][:5]])" >> $out
    tail -1 $out
  done
done
