# round 6: O-emission placement A/B (V1 stores in the core, V2 parked in dO rows + stored after the dxn GEMM = product,
# V3 parked + stored between the dW and dxn GEMMs); SLP variants F (fenced Lp) / G (Li loaded in the pixel loop)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r6g_twh_o_ab.txt
for rep in 1 2; do
  for v in ov1 prod ov3; do
    lib=cesm_emulator_amd/libcesm_hip_$v.so; [ $v = prod ] && lib=cesm_emulator_amd/libcesm_hip.so
    echo -n "$v: " >> gpurun_out/r6g_twh_o_ab.txt
    CESM_HIP_LIB=$lib timeout -k 10 200 python3 tools/twh_o_time.py 8 10 2>/dev/null | tail -1 >> gpurun_out/r6g_twh_o_ab.txt
  done
done
cat gpurun_out/r6g_twh_o_ab.txt
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "tblock_fold or nan" > gpurun_out/r6g_pytest.log 2>&1
tail -1 gpurun_out/r6g_pytest.log
for v in F G; do
  CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_slp$v.so timeout -k 10 150 python3 tools/slp_region_check.py > gpurun_out/r6g_slp_$v.txt 2>&1
  echo "$v: $(grep -c 'dx 0,' gpurun_out/r6g_slp_$v.txt) of 9 calls repeatable"
done
