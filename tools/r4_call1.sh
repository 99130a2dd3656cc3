#!/bin/bash
# Round 4, first GPU call: the new full-size tests (tflash F=120 at 192x288, config 4 / 5 per-GPU legs) and the
# CESM_WGRAD_STREAM=1 diagnostic (per-step wall + allocator counters, then a kernel trace).
set -e
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_tflash_long_window_full_grid" \
  "tests/test_gpu_kernels.py::test_temporal_attention_core" \
  "tests/test_gpu_prod_parity.py::test_decadal_window_full_grid_bf16_step_repeatable" \
  "tests/test_gpu_prod_parity.py::test_full_grid_bf16_batch5_split" -s > gpurun_out/r4c1_pytest.log 2>&1
tail -3 gpurun_out/r4c1_pytest.log
CESM_WGRAD_STREAM=0 timeout -k 10 200 python3 -u tools/wgrad_stream_diag.py 4 > gpurun_out/r4c1_ws0.txt 2>&1
CESM_WGRAD_STREAM=1 timeout -k 10 200 python3 -u tools/wgrad_stream_diag.py 4 > gpurun_out/r4c1_ws1.txt 2>&1
cat gpurun_out/r4c1_ws0.txt gpurun_out/r4c1_ws1.txt
CESM_WGRAD_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r4c1_prof -o run -- \
  python3 tools/wgrad_stream_diag.py 3 > gpurun_out/r4c1_prof.log 2>&1
python3 tools/trace_gaps.py gpurun_out/r4c1_prof 25 > gpurun_out/r4c1_ws1_gaps.txt
rm -rf gpurun_out/r4c1_prof
head -40 gpurun_out/r4c1_ws1_gaps.txt
