# round 6: O emitted by the temporal backward instead of the forward -- micro timing, parity tests, bench
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/twh_o_time.py 8 10 > gpurun_out/r6f_twh_o_time.txt 2>&1
cat gpurun_out/r6f_twh_o_time.txt | tail -2
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_determinism.py tests/test_gpu_stale_state.py tests/test_gpu_prod_parity.py > gpurun_out/r6f_pytest.log 2>&1
tail -2 gpurun_out/r6f_pytest.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-configs '' > gpurun_out/r6f_bench.json 2> gpurun_out/r6f_bench.err
python3 -c "import json; d=json.load(open('gpurun_out/r6f_bench.json')); print(d['value'], d['ms_per_step'])"
