#!/bin/bash
# k_xattn_seg grid A/B at 1 / 2 / 4 windows (tuning build: WHISPER_HIP_XS_K per launch; -n = n workgroups)
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export WHISPER_HIP_LIB=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
timeout -k 10 300 python3 -u profiles/xattn_probe.py large-v3 1,2,4 0,-20,-40,-80,-120,-160,0 > gpurun_out/xattn_grid_${tag}.txt 2>&1 || exit 2
cat gpurun_out/xattn_grid_${tag}.txt
