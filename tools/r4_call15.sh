#!/bin/bash
# Round-4 call 15: warp-specialized conv items in per-XCD column runs (libcesm_hip_wsCM.so) vs the default order: bit
# check + level-0 tests with the variant, main-leg bench A/B.  tools/r4_call15.sh <tag>
set -e
tag=${1:-r4c15}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/${tag}_md5.txt
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_wsCM.so timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q \
  -k "conv3x3p or gn_epilogue or concurrent" --timeout 240 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
tail -2 gpurun_out/${tag}_pytest.log
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_wsCM.so timeout -k 10 300 python3 -u tools/ws_check.py > gpurun_out/${tag}_ws_cm.txt 2>&1 || true
head -3 gpurun_out/${tag}_ws_cm.txt | tail -1; grep "(96, 192, 288, 64, 0, 64)" gpurun_out/${tag}_ws_cm.txt || true
out=gpurun_out/${tag}_bench_ab.txt
: > $out
for rep in 1 2; do
  for v in default wsCM; do
    lib=cesm_emulator_amd/libcesm_hip.so; [ $v != default ] && lib=cesm_emulator_amd/libcesm_hip_$v.so
    CESM_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" \
      > gpurun_out/${tag}_b.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/${tag}_b.json')); print('$v', d['value'], d['ms_per_step'], [(t['kernel'], t['avg_us']) for t in d['top_kernels'][:6]])" >> $out
  done
done
cat $out
