# round 6: batched weight re-pack timing + test
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/pack_time.py 20 > gpurun_out/r6n_pack_time.txt 2>&1; tail -1 gpurun_out/r6n_pack_time.txt
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "pack_batch" > gpurun_out/r6n_pytest.log 2>&1
tail -1 gpurun_out/r6n_pytest.log
