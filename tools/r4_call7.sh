#!/bin/bash
# Round-4 call 7: L2 touch prefetch in the warp-specialized conv (default lib) vs without (libcesm_hip_wsT0.so), and
# in the halo conv (libcesm_hip_h3T.so): conv bit check + timing per lib, conv GPU tests, main-leg bench A/B.
set -e
tag=${1:-r4c7}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "conv3x3p or gn_epilogue or whole_net or decadal_window_full" \
  --timeout 240 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
tail -2 gpurun_out/${tag}_pytest.log
timeout -k 10 300 python3 -u tools/ws_check.py > gpurun_out/${tag}_ws_touch.txt 2>&1 || true
tail -9 gpurun_out/${tag}_ws_touch.txt
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_wsT0.so timeout -k 10 300 python3 -u tools/ws_check.py > gpurun_out/${tag}_ws_notouch.txt 2>&1 || true
tail -9 gpurun_out/${tag}_ws_notouch.txt
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_h3T.so timeout -k 10 300 python3 -u tools/ws_check.py > gpurun_out/${tag}_ws_h3touch.txt 2>&1 || true
tail -9 gpurun_out/${tag}_ws_h3touch.txt
out=gpurun_out/${tag}_bench_ab.txt
: > $out
for rep in 1 2; do
  for v in default wsT0 h3T wgT; do
    lib=cesm_emulator_amd/libcesm_hip.so; [ $v != default ] && lib=cesm_emulator_amd/libcesm_hip_$v.so
    CESM_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" \
      > gpurun_out/${tag}_b.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/${tag}_b.json')); print('$v', d['value'], d['ms_per_step'])" >> $out
  done
done
cat $out
