#!/bin/bash
# Round-4 call 9: resident weights in the warp-specialized level-0 conv (default) vs not (libcesm_hip_wsNoRW.so), and the
# w36 wgrad touch (libcesm_hip_w36T.so): conv GPU tests, conv bit check + timing, main-leg bench A/B.
set -e
tag=${1:-r4c9}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q -k "conv3x3p or gn_epilogue or whole_net or decadal_window or concurrent" \
  --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
tail -2 gpurun_out/${tag}_pytest.log
timeout -k 10 300 python3 -u tools/ws_check.py > gpurun_out/${tag}_ws_rw.txt 2>&1 || true
tail -9 gpurun_out/${tag}_ws_rw.txt
out=gpurun_out/${tag}_bench_ab.txt
: > $out
for rep in 1 2; do
  for v in default wsNoRW w36T; do
    lib=cesm_emulator_amd/libcesm_hip.so; [ $v != default ] && lib=cesm_emulator_amd/libcesm_hip_$v.so
    CESM_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" \
      > gpurun_out/${tag}_b.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/${tag}_b.json')); print('$v', d['value'], d['ms_per_step'], [(t['kernel'], t['avg_us']) for t in d['top_kernels'][:6]])" >> $out
  done
done
cat $out
