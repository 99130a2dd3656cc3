# round 6: kernel profile of the current tree + A/B: C = 128 fused temporal block with O from the backward
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# (profile taken in the first r6i call)
: > gpurun_out/r6i_o128_ab.txt
for rep in 1 2; do
  for v in - TBLOCK_FWD_O_MAXC=64; do
    timeout -k 10 300 python3 tools/vn_const_ab.py $v --steps 20 --warmup 5 --no-cpu-baseline --other-configs '' 2>> gpurun_out/r6i_o128_ab.err >> gpurun_out/r6i_o128_ab.txt
    tail -1 gpurun_out/r6i_o128_ab.txt
  done
done
