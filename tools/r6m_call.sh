# round 6: sized batched weight pack (test + whole-step A/B against the previous pack kernel) + SQ passes
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "pack_batch or conv_fwd_bwd" tests/test_gpu_train.py > gpurun_out/r6m_pytest.log 2>&1
tail -1 gpurun_out/r6m_pytest.log
bash tools/gpu_call.sh r6m prof
bash tools/gpu_call.sh r6m sq:wgrad3x3c64,wgrad3x3w36c64,conv3x3ws,gn_bwd_apply,gn_apply,slaf_out
