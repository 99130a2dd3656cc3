# round 6: square-tile 1x1 wgrad -- test, micro timing (default and without), whole-step and F = 120 A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > gpurun_out/r6s_pytest.log 2>&1
tail -1 gpurun_out/r6s_pytest.log
timeout -k 10 300 python3 tools/wgrad_vs_blas.py > gpurun_out/r6s_wgrad_sq.txt 2>&1
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_sqoff.so timeout -k 10 300 python3 tools/wgrad_vs_blas.py > gpurun_out/r6s_wgrad_sqoff.txt 2>&1
paste -d'\n' gpurun_out/r6s_wgrad_sq.txt gpurun_out/r6s_wgrad_sqoff.txt | grep -v amdgpu | cut -c1-90
bash tools/gpu_call.sh r6s ab:sqoff
BENCH_ARGS="--frames 120 --batch 1" bash tools/gpu_call.sh r6s120 ab:sqoff
