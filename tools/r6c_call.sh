set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 -k "qkv_bwd or temporal_attention_core or tflash or decadal or determinism or stale" > gpurun_out/r6c_pytest.log 2>&1 || { tail -30 gpurun_out/r6c_pytest.log; exit 1; }
tail -2 gpurun_out/r6c_pytest.log
timeout -k 10 300 python3 tools/qkv_bwd_time.py > gpurun_out/r6c_qkv_time.txt 2>&1; cat gpurun_out/r6c_qkv_time.txt | grep -v amdgpu.ids
for lib in default prepk default prepk; do
  l=""; [ $lib = prepk ] && l=cesm_emulator_amd/libcesm_hip_prepk.so
  echo "== $lib" >> gpurun_out/r6c_tflash_ab.txt
  CESM_HIP_LIB=$l timeout -k 10 120 python3 tools/tflash_time.py 120 192 288 1 3 1 >> gpurun_out/r6c_tflash_ab.txt 2>&1
done
grep -v amdgpu.ids gpurun_out/r6c_tflash_ab.txt
BENCH_ARGS="--frames 120 --batch 1" bash tools/gpu_call.sh r6c ab:prepk
