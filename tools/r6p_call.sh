# round 6: twh_bwd O stores paired to 16 B by permlane16 swaps -- micro timing + fold test
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/twh_o_time.py 8 10 > gpurun_out/r6p_twh_o_time.txt 2>&1; tail -1 gpurun_out/r6p_twh_o_time.txt
timeout -k 10 200 python3 tools/twh_o_time.py 8 10 2>&1 | tail -1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "tblock_fold" > gpurun_out/r6p_pytest.log 2>&1
tail -1 gpurun_out/r6p_pytest.log
