# round 6: square-tile wgrad with 64-row tiles (the level-0 to_out) -- test + micro
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "wgrad" > gpurun_out/r6t_pytest.log 2>&1
tail -1 gpurun_out/r6t_pytest.log
timeout -k 10 300 python3 tools/wgrad_vs_blas.py 2>&1 | grep -v amdgpu | cut -c1-100
