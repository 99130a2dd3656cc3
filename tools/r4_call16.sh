#!/bin/bash
# Round-4 call 16: halo conv two-phase chunk wait (libcesm_hip_h3s.so, -DH3_SPLIT=1) vs the default: bit
# check + level-0 tests with the variant, main-leg bench A/B.  tools/r4_call16.sh <tag>
set -e
tag=${1:-r4c16}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_h3s.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q \
  -k "conv and not wgrad" --timeout 240 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
tail -2 gpurun_out/${tag}_pytest.log
timeout -k 10 400 python3 -u tools/conv_lib_ab.py cesm_emulator_amd/libcesm_hip.so cesm_emulator_amd/libcesm_hip_h3s.so \
  > gpurun_out/${tag}_conv_ab.txt 2>&1 || true
grep -v amdgpu.ids gpurun_out/${tag}_conv_ab.txt | tail -10
out=gpurun_out/${tag}_bench_ab.txt
: > $out
for rep in 1 2; do
  for v in default h3s; do
    lib=cesm_emulator_amd/libcesm_hip.so; [ $v != default ] && lib=cesm_emulator_amd/libcesm_hip_$v.so
    CESM_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" \
      > gpurun_out/${tag}_b.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/${tag}_b.json')); print('$v', d['value'], d['ms_per_step'], [(t['kernel'], t['avg_us']) for t in d['top_kernels'][:6]])" >> $out
  done
done
cat $out
