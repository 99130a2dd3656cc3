# round 6: unused-half packed-fp32 probe + bench of the O-from-backward tree
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -fno-slp-vectorize tools/diag/pk_unused_half_probe.hip -o /tmp/pk_unused_half_probe 2>/dev/null
timeout -k 10 60 /tmp/pk_unused_half_probe > gpurun_out/r6h_pk_unused_half.txt 2>&1
cat gpurun_out/r6h_pk_unused_half.txt | tail -12
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-configs '' > gpurun_out/r6h_bench.json 2> gpurun_out/r6h_bench.err
python3 -c "import json; d=json.load(open('gpurun_out/r6h_bench.json')); print(d['value'], d['ms_per_step'])"
