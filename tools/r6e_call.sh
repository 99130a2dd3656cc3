# round 6: SLP variant E (pixel loop of twh_bwd not unrolled, SLP on) + the fused forwards' O-write cost
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CESM_HIP_LIB=cesm_emulator_amd/libcesm_hip_slpE.so timeout -k 10 150 python3 tools/slp_region_check.py > gpurun_out/r6e_slp_E.txt 2>&1
grep -c "dx 0," gpurun_out/r6e_slp_E.txt || true
timeout -k 10 200 python3 tools/fwd_o_cost.py 8 20 > gpurun_out/r6e_fwd_o_cost.txt 2>&1
cat gpurun_out/r6e_fwd_o_cost.txt
