#!/bin/bash
# tuning-library A/B of the 100-row step tail: the selection's slice count (WHISPER_HIP_LP_NS)
# and k_vocab_2p's weight chunks in flight (WHISPER_HIP_V2P_DEPTH); step graph ms, alternated
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "0 2" "16 2" "32 2" "0 3"; do
    set -- $cfg
    WHISPER_HIP_LIB=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so WHISPER_HIP_LP_NS=$1 WHISPER_HIP_V2P_DEPTH=$2 \
      timeout -k 10 200 python3 profiles/step_profile.py --windows 20 --steps 32 | sed "s/^/ns $1 depth $2: /" >> gpurun_out/tail_ab_${tag}.txt 2>&1 || exit 1
  done
done
cat gpurun_out/tail_ab_${tag}.txt
