#!/bin/bash
# Single-window encoder A/B (round 4): the residual GEMMs' two-way in-launch K split
# (k_gemm_tile KZ = 2, default) vs one workgroup per tile (WHISPER_HIP_ENC_KZ=0, tuning
# library), profiles/enc_chunk_probe.py --windows 1, alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export WHISPER_HIP_LIB=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for i in 1 2; do
  for kz in 1 0; do
    echo "WHISPER_HIP_ENC_KZ=$kz"
    WHISPER_HIP_ENC_KZ=$kz timeout -k 10 240 python3 profiles/enc_chunk_probe.py --windows 1 --reps 20 || exit 1
  done
done
