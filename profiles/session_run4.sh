#!/bin/bash
# GPU suite + encoder chunk A/B (tuning library) + step profile + default bench
#   profiles/session_run4.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_${tag}.log 2>&1 || { tail -30 gpurun_out/gpu_tests_${tag}.log; exit 1; }
tail -3 gpurun_out/gpu_tests_${tag}.log
for c in 16 20 10 7; do
  WHISPER_HIP_LIB=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so WHISPER_HIP_ENC_CHUNK=$c \
    timeout -k 10 200 python3 profiles/enc_chunk_probe.py >> gpurun_out/enc_chunk_${tag}.txt 2>&1 || exit 6
done
cat gpurun_out/enc_chunk_${tag}.txt
bash profiles/profile_step.sh w20_${tag} --windows 20 --steps 16 --encode 4 || exit 2
head -3 gpurun_out/step_w20_${tag}_plain.txt
grep -E 'attn_enc|gemm_256|layernorm' gpurun_out/step_w20_${tag}_summary.txt
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${tag}.json 2> gpurun_out/bench_${tag}.err || exit 4
cat gpurun_out/bench_${tag}.json
