# round 6 vs round 5 final tree (1151c7a, checked out under r5tree/), same box, alternating, twice: the headline step
# and the F = 120 leg
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/r6l_r5_vs_r6.txt
for rep in 1 2; do
  for t in r5tree .; do
    (cd $t && timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --other-configs '' 2>/dev/null) > gpurun_out/r6l_tmp.json
    python3 -c "import json; d=json.load(open('gpurun_out/r6l_tmp.json')); print('$t', 'F12 B8', d['value'], d['ms_per_step'])" >> gpurun_out/r6l_r5_vs_r6.txt
    tail -1 gpurun_out/r6l_r5_vs_r6.txt
  done
done
for rep in 1 2; do
  for t in r5tree .; do
    (cd $t && timeout -k 10 300 python3 bench.py --frames 120 --batch 1 --steps 10 --warmup 3 --no-cpu-baseline --no-probe --other-configs '' 2>/dev/null) > gpurun_out/r6l_tmp.json
    python3 -c "import json; d=json.load(open('gpurun_out/r6l_tmp.json')); print('$t', 'F120 B1', d['value'], d['ms_per_step'])" >> gpurun_out/r6l_r5_vs_r6.txt
    tail -1 gpurun_out/r6l_r5_vs_r6.txt
  done
done
