bash tools/gpu_check.sh r3c r2; rc=$?
if [ $rc -le 1 ]; then
  CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_slp.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_determinism.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3c_slp_det.log 2>&1
  echo "slp determinism rc=$?"
fi
exit $rc
