#!/bin/bash
# step cross-attention grid at few windows (tuning library, WHISPER_HIP_XS_K: 0 = default,
# -n = spread over n workgroups): the single-window latency path
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  WHISPER_HIP_LIB=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so \
    timeout -k 10 300 python3 profiles/xattn_probe.py large-v3 1,2,4 0,-40,-80,-120,-160,-200,-256 >> gpurun_out/xgrid_${tag}.txt 2>&1 || exit 1
done
cat gpurun_out/xgrid_${tag}.txt
