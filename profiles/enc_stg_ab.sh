#!/bin/bash
# Encoder A/B (round 4): k_gemm_tile's 128 x 64 tiles with three register sets of staged
# global loads (WHISPER_HIP_GEMM_STG=3) vs two (2), tuning library, one window and 20
# windows (profiles/enc_chunk_probe.py), alternated twice; then a kernel trace of each
# single-window form (outputs under gpurun_out/enc_stg_*).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export WHISPER_HIP_LIB=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
for i in 1 2; do
  for s in 3 2; do
    for w in 1 20; do
      echo "WHISPER_HIP_GEMM_STG=$s"
      WHISPER_HIP_GEMM_STG=$s timeout -k 10 240 python3 profiles/enc_chunk_probe.py --windows $w --reps 10 || exit 1
    done
  done
done
for s in 3 2; do
  WHISPER_HIP_GEMM_STG=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/enc_stg_prof$s -o run -- \
    python3 profiles/enc_chunk_probe.py --windows 1 --reps 10 > gpurun_out/enc_stg_prof$s.log 2>&1 || exit 1
done
for s in 3 2; do
  db=$(ls gpurun_out/enc_stg_prof$s/*/run_results.db gpurun_out/enc_stg_prof$s/run_results.db 2>/dev/null | head -1)
  python3 profiles/summarize_db.py $db 20 gpurun_out/enc_stg_$s.csv > gpurun_out/enc_stg_summary$s.txt
done
