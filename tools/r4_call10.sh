#!/bin/bash
# Round-4 call 10: halo-conv weight chunk through registers (libcesm_hip_h3W.so) vs LDS-DMA (default): halo-conv bit
# check + timing, main-leg bench A/B.  tools/r4_call10.sh <tag>
set -e
tag=${1:-r4c10}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_h3W.so timeout -k 10 300 python3 -u tools/ws_check.py > gpurun_out/${tag}_ws_h3w.txt 2>&1 || true
tail -9 gpurun_out/${tag}_ws_h3w.txt
out=gpurun_out/${tag}_bench_ab.txt
: > $out
for rep in 1 2; do
  for v in default h3W; do
    lib=cesm_emulator_amd/libcesm_hip.so; [ $v != default ] && lib=cesm_emulator_amd/libcesm_hip_$v.so
    CESM_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" \
      > gpurun_out/${tag}_b.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/${tag}_b.json')); print('$v', d['value'], d['ms_per_step'], [(t['kernel'], t['avg_us']) for t in d['top_kernels'][:6]])" >> $out
  done
done
cat $out
