#!/bin/bash
# One GPU-box session driver (replaces the round-1..3 one-off session_run*.sh scripts).
#   profiles/gpu_session.sh <tag> <step> [<step> ...]
# steps (each under its own time limit; the first failure ends the session):
#   tests      python -m pytest tests -m gpu (thread timeouts, one process)
#   smoke      __graft_entry__.smoke()
#   cfg3       bench.py default (config 3, with the CPU baseline)
#   cfg3q      bench.py default without the CPU baseline
#   cfg2       turbo, one 30 s window
#   cfg5       word timestamps
#   cfg4       one 3600 s file through the sharded path, --verify 1 (N = 1)
#   profeager  rocprofv3 --kernel-trace --stats of bench.py in eager mode (tuning library,
#              WHISPER_HIP_EAGER=1: a graph-mode bench dispatches ~80k graph kernels, past the
#              point where rocprofv3's kernel trace segfaults)
#   step20 / step1 / stepturbo   graph-mode step profile (profiles/profile_step.sh)
#   pmc        PMC traffic passes (profiles/pmc_pass.sh)
#   ab:<VAR>   xattn_probe step graphs at 1 / 20 windows with the tuning library, VAR=1 vs VAR=0, twice
# outputs: gpurun_out/<step>_<tag>.*
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out
TUNE=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
    tests)
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > $O/tests_${tag}.txt 2>&1 || { tail -30 $O/tests_${tag}.txt; exit 2; }
      tail -3 $O/tests_${tag}.txt ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_${tag}.txt 2>&1 || exit 3
      cat $O/smoke_${tag}.txt ;;
    cfg3)
      timeout -k 10 500 python3 bench.py > $O/cfg3_${tag}.json 2> $O/cfg3_${tag}.err || exit 4
      cat $O/cfg3_${tag}.json ;;
    cfg3q)
      timeout -k 10 300 python3 bench.py --cpu-baseline 0 > $O/cfg3q_${tag}.json 2> $O/cfg3q_${tag}.err || exit 4
      cat $O/cfg3q_${tag}.json ;;
    cfg2)
      timeout -k 10 300 python3 bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 \
        > $O/cfg2_${tag}.json 2> $O/cfg2_${tag}.err || exit 5
      cat $O/cfg2_${tag}.json ;;
    cfg5)
      timeout -k 10 400 python3 bench.py --word-timestamps 1 --cpu-baseline 0 > $O/cfg5_${tag}.json 2> $O/cfg5_${tag}.err || exit 6
      cat $O/cfg5_${tag}.json ;;
    cfg4)
      timeout -k 10 500 python3 bench.py --sharded-file 1 --seconds 3600 --verify 1 --cpu-baseline 0 --steps 1 \
        > $O/cfg4_${tag}.json 2> $O/cfg4_${tag}.err || exit 7
      cat $O/cfg4_${tag}.json ;;
    profeager)
      WHISPER_HIP_LIB=$TUNE WHISPER_HIP_EAGER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/profeager_${tag} -o run -- \
        python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --latency 0 > $O/profeager_${tag}.log 2>&1 || exit 9 ;;
    step20) bash profiles/profile_step.sh w20_${tag} --model large-v3 --windows 20 || exit 10 ;;
    step1) bash profiles/profile_step.sh w1_${tag} --model large-v3 --windows 1 || exit 11 ;;
    stepturbo) bash profiles/profile_step.sh turbo1_${tag} --model turbo --windows 1 || exit 12 ;;
    pmc) bash profiles/pmc_pass.sh ${tag} || exit 13 ;;
    ab:*)
      var=${step#ab:}
      out=$O/ab_${var}_${tag}.txt
      : > $out
      for rep in 1 2; do
        for v in 1 0; do
          echo "$var=$v" >> $out
          env WHISPER_HIP_LIB=$TUNE $var=$v timeout -k 10 200 python3 -u profiles/xattn_probe.py large-v3 1,20 0 >> $out 2>&1 || exit 14
        done
      done
      cat $out ;;
    *) echo "unknown step $step"; exit 1 ;;
  esac
done
