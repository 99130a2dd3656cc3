# round 6 evidence call: SLP region bisection, F = 120 fused-qkv A/B (dispatch constant), PMC traffic, SQ passes
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in S A B C D; do
  CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_slp$v.so timeout -k 10 150 python3 tools/slp_region_check.py > gpurun_out/r6d_slp_$v.txt 2>&1
  tail -4 gpurun_out/r6d_slp_$v.txt | cut -c1-150
done
: > gpurun_out/r6d_qkv_f120_ab.txt
for rep in 1 2; do
  for maxc in 64 0; do
    timeout -k 10 300 python3 -c "
import runpy, sys
import cesm_emulator_amd.video_net as V
V.QKV_BWD_MAXC = $maxc
sys.argv = ['bench.py', '--frames', '120', '--batch', '1', '--steps', '10', '--warmup', '3', '--no-cpu-baseline', '--no-probe', '--other-configs', '']
runpy.run_path('bench.py', run_name='__main__')" 2>> gpurun_out/r6d_qkv_f120_ab.err | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('QKV_BWD_MAXC=$maxc', d['value'], d['ms_per_step'])" >> gpurun_out/r6d_qkv_f120_ab.txt
    tail -1 gpurun_out/r6d_qkv_f120_ab.txt
  done
done
bash tools/gpu_call.sh r6d traffic sq:twh_bwd,slah_dx,tw_fwd,conv3x3_bf16,qkv_bwd
