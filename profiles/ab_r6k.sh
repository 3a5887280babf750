# Round 6 (k): the step self-attention with coalesced K reads (PIPE 3, WHISPER_HIP_SA_KCO=1,
# tuning build default) vs the lane-per-key K reads (PIPE 1, KCO=0): the GPU parity suites
# that run the step self-attention on the tuning build, then chain traces at 0 and 150
# replayed steps (context ~12 and ~160 tokens), alternated, one box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
N=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so
WHISPER_HIP_LIB=$N timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_batch.py tests/test_gpu_models.py > gpurun_out/kco_tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for adv in 0 150; do
    for v in 1 0; do
      WHISPER_HIP_LIB=$N WHISPER_HIP_SA_KCO=$v timeout -k 10 150 python profiles/chain_trace.py 20 8 $adv > gpurun_out/ctk_${v}_${adv}_$rep.txt 2>&1 || exit 2
    done
  done
done
for v in 1 0; do
  WHISPER_HIP_LIB=$N WHISPER_HIP_SA_KCO=$v timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/kco_c3_$v.json 2>/dev/null || exit 3
  WHISPER_HIP_LIB=$N WHISPER_HIP_SA_KCO=$v timeout -k 10 300 python bench.py --model turbo --seconds 30 --max-windows 1 --cpu-baseline 0 > gpurun_out/kco_c2_$v.json 2>/dev/null || exit 4
done
