#!/bin/bash
# conv3x3p single tap loop + static split: tests, kernel summary of the bench step, WGRAD_STREAM probe A/B
set -e
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > gpurun_out/r4c2_md5.txt
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_prod_parity.py tests/test_gpu_kernels.py tests/test_gpu_determinism.py \
  -k "conv3x3p or gn_epilogue or whole_net or tblock or fused_temporal or repeat or determin" > gpurun_out/r4c2_pytest.log 2>&1
tail -2 gpurun_out/r4c2_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4c2_prof -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --other-configs "" > gpurun_out/r4c2_prof.json 2> gpurun_out/r4c2_prof.err
python3 tools/kstats.py gpurun_out/r4c2_prof 7 40 > gpurun_out/r4c2_kernel_summary.txt
rm -rf gpurun_out/r4c2_prof
head -14 gpurun_out/r4c2_kernel_summary.txt
for v in "CESM_WGRAD_STREAM=0" "CESM_WGRAD_STREAM=1"; do
  for pr in "" "--no-probe"; do
    env $v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --other-configs "" $pr 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '$pr', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r4c2_ws_probe_ab.txt
  done
done
BENCH_VARIANTS="r4base r4fold" bash tools/r4_call3.sh r4c3 r4base r4k16nb r4k16 r4k16pg2 r4nnan r4fold
