#!/bin/bash
# One entry point for the gpurun calls of a round (replaces round 4's per-call r4_call*.sh scripts):
#   tools/gpu_call.sh <tag> <step> [<step> ...]
# Steps (run in order; each GPU step has its own time limit, the first failure ends the call):
#   test[:<pytest -k expr>]   pytest -m gpu (optionally -k)              -> gpurun_out/<tag>_pytest.log
#   smoke                      __graft_entry__.smoke()                    -> gpurun_out/<tag>_smoke.log
#   bench                      bench.py, the default contract run         -> gpurun_out/<tag>_bench.json
#   prof                       rocprofv3 --kernel-trace --stats of the headline step -> <tag>_kernel_summary.txt
#   calls:<pattern>            per-call durations of kernels matching <pattern> in the headline step
#   f120                       the F = 120 leg profiled (kernel totals + per-call tflash)
#   traffic                    PMC HBM traffic of one step -> profiles/step_traffic.json
#   sq:<k1,k2,..>              SQ counter passes over one step for the named kernels
#   ab:<v1,v2,..>              whole-step A/B: default library vs libcesm_hip_<v>.so, alternating, twice
#   envab:<ENV=a|ENV=b|..>     whole-step A/B over environment settings ("-" = default), twice
#   tb:<v1,v2,..>              fused attention block micro-timing (tools/tblock_time.py), default vs variants
#   py:<script args..>         any tools/ python script (spaces as '+'), e.g. py:ws_check.py
#   run:<name>:<cmd..>         any command (spaces as '+') with a 600 s limit -> gpurun_out/<tag>_<name>.txt
# Extra bench arguments for ab/envab/prof/calls: BENCH_ARGS="--frames 120 --batch 1" tools/gpu_call.sh ...
set -e
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
cd "$root"
mkdir -p gpurun_out
md5sum cesm_emulator_amd/*.so > "gpurun_out/${tag}_md5.txt"
bargs=${BENCH_ARGS:-}
lib() { if [ "$1" = default ]; then echo ""; else echo "cesm_emulator_amd/libcesm_hip_$1.so"; fi; }
for step in "$@"; do
  kind=${step%%:*}; arg=""; [ "$kind" != "$step" ] && arg=${step#*:}
  case $kind in
    test)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q "${k[@]}" --timeout 400 --timeout-method thread \
        > "gpurun_out/${tag}_pytest.log" 2>&1
      tail -2 "gpurun_out/${tag}_pytest.log";;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${tag}_smoke.log" 2>&1
      tail -2 "gpurun_out/${tag}_smoke.log";;
    bench)
      timeout -k 10 600 python3 bench.py > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.err"
      python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], {k: v.get('ms_per_step') for k, v in d.get('other_configs', {}).items()})";;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof" -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --other-configs "" $bargs \
        > "gpurun_out/${tag}_prof.json" 2> "gpurun_out/${tag}_prof.err"
      python3 tools/kstats.py "gpurun_out/${tag}_prof" 7 70 > "gpurun_out/${tag}_kernel_summary.txt"
      rm -rf "gpurun_out/${tag}_prof"
      head -14 "gpurun_out/${tag}_kernel_summary.txt";;
    calls)
      timeout -k 10 300 rocprofv3 --kernel-trace -d "gpurun_out/${tag}_calls" -o run -- \
        python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-probe --other-configs "" $bargs \
        > "gpurun_out/${tag}_calls.json" 2> "gpurun_out/${tag}_calls.err"
      python3 tools/kcalls.py "gpurun_out/${tag}_calls" "$arg" 2000 > "gpurun_out/${tag}_calls.txt"
      rm -rf "gpurun_out/${tag}_calls"
      wc -l "gpurun_out/${tag}_calls.txt";;
    f120)
      timeout -k 10 400 rocprofv3 --kernel-trace -d "gpurun_out/${tag}_f120" -o run -- \
        python3 bench.py --frames 120 --batch 1 --steps 2 --warmup 1 --no-cpu-baseline --no-probe --other-configs "" \
        > "gpurun_out/${tag}_f120.json" 2> "gpurun_out/${tag}_f120.err"
      python3 tools/kstats.py "gpurun_out/${tag}_f120" 3 45 > "gpurun_out/${tag}_f120_summary.txt"
      python3 tools/kcalls.py "gpurun_out/${tag}_f120" tflash 40 > "gpurun_out/${tag}_f120_tflash_calls.txt"
      rm -rf "gpurun_out/${tag}_f120"
      head -16 "gpurun_out/${tag}_f120_summary.txt";;
    traffic)
      bash tools/pmc_traffic.sh "${tag}" > "gpurun_out/${tag}_traffic.log" 2>&1
      tail -3 "gpurun_out/${tag}_traffic.log";;
    sq)
      PMC_KERNELS="${arg//,/ }" bash tools/pmc_step_sq.sh "${tag}" > "gpurun_out/${tag}_sq.log" 2>&1
      tail -3 "gpurun_out/${tag}_sq.log";;
    ab)
      out=gpurun_out/${tag}_bench_ab.txt; : > "$out"
      for rep in 1 2; do
        for v in default ${arg//,/ }; do
          CESM_HIP_LIB=$(lib "$v") timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --other-configs "" \
            --steps 10 --warmup 3 $bargs 2>> "gpurun_out/${tag}_bench_ab.err" | \
            python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d.get('loss'))" >> "$out"
          tail -1 "$out"
        done
      done;;
    envab)
      out=gpurun_out/${tag}_env_ab.txt; : > "$out"
      IFS='|' read -r -a settings <<< "$arg"
      for rep in 1 2; do
        for v in "${settings[@]}"; do
          envs=""; [ "$v" != "-" ] && envs="$v"
          env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-probe --other-configs "" \
            --steps 10 --warmup 3 $bargs 2>> "gpurun_out/${tag}_env_ab.err" | \
            python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" >> "$out"
          tail -1 "$out"
        done
      done;;
    tb)
      out=gpurun_out/${tag}_tb.txt; : > "$out"
      for rep in 1 2; do
        for v in default ${arg//,/ }; do
          echo "== $v" >> "$out"
          CESM_HIP_LIB=$(lib "$v") timeout -k 10 150 python3 tools/tblock_time.py 64 10 >> "$out" 2>&1
          tail -1 "$out"
        done
      done;;
    py)
      timeout -k 10 400 python3 tools/${arg//+/ } > "gpurun_out/${tag}_$(echo "${arg%%+*}" | tr -c 'a-zA-Z0-9_\n' _).txt" 2>&1
      tail -5 "gpurun_out/${tag}_$(echo "${arg%%+*}" | tr -c 'a-zA-Z0-9_\n' _).txt";;
    run)
      name=${arg%%:*}; cmd=${arg#*:}
      timeout -k 10 600 ${cmd//+/ } > "gpurun_out/${tag}_${name}.txt" 2>&1
      tail -3 "gpurun_out/${tag}_${name}.txt";;
    *) echo "unknown step $step"; exit 2;;
  esac
done
