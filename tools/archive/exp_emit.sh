set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for e in 1 0; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/exp1_sla$e -o run -- python3 tools/sla_micro.py 3 $e > gpurun_out/exp1_sla$e.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/exp1_tb$e -o run -- python3 tools/tblock_micro.py 64 3 $e > gpurun_out/exp1_tb$e.log 2>&1
done
