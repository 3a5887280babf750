# Round 6 (l): k_vocab_1p (one pass over K, WHISPER_HIP_V1P) and the coalesced-K self-attention
# from 64 cached keys on (WHISPER_HIP_SA_KCO / _KCO_MIN) against round 6's shipped forms
# (V1P=0, KCO=0): parity suites on the shipped library (new defaults), then chain traces at 0
# and 150 replayed steps and config 3 / 2 bench lines on the tuning build, alternated.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch.py tests/test_gpu_models.py tests/test_gpu_tail.py > gpurun_out/l_tests.txt 2>&1 || exit 1
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for rep in 1 2; do
  for adv in 0 150; do
    for v in old new vocab; do
      case $v in old) E="WHISPER_HIP_V1P=0 WHISPER_HIP_SA_KCO=0";; new) E="";; vocab) E="WHISPER_HIP_SA_KCO=0";; esac
      env $E WHISPER_HIP_LIB=$N timeout -k 10 150 python profiles/chain_trace.py 20 8 $adv > gpurun_out/ctl_${v}_${adv}_$rep.txt 2>&1 || exit 2
    done
  done
done
for v in new old; do
  case $v in old) E="WHISPER_HIP_V1P=0 WHISPER_HIP_SA_KCO=0";; new) E="";; esac
  env $E WHISPER_HIP_LIB=$N timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/l_c3_$v.json 2>/dev/null || exit 3
  env $E WHISPER_HIP_LIB=$N timeout -k 10 300 python bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 > gpurun_out/l_c2_$v.json 2>/dev/null || exit 4
done
