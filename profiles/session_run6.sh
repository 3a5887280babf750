#!/bin/bash
# k_gemm_256 16x16x32 vs 32x32x16 MFMA A/B: isolated shapes (tools/gemm_bench 256 vs 257) and
# the whole encoder through the tuning library (WHISPER_HIP_GEMM=257)
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 240 ./whisper.coreml_amd/tools/gemm_bench 16 7 256 257 > gpurun_out/gemm_mf_${tag}.txt 2>&1 || { cat gpurun_out/gemm_mf_${tag}.txt; exit 1; }
cat gpurun_out/gemm_mf_${tag}.txt
for sel in 256 257 256 257; do
  WHISPER_HIP_LIB=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so WHISPER_HIP_GEMM=$sel \
    timeout -k 10 200 python3 profiles/enc_chunk_probe.py | sed "s/^/gemm $sel: /" >> gpurun_out/enc_mf_${tag}.txt 2>&1 || exit 2
done
cat gpurun_out/enc_mf_${tag}.txt
