#!/bin/bash
# k_resid_ln thread shape A/B: step graph at 1 / 20 windows (tuning build: WHISPER_HIP_RLN_256=1 = round-3 form)
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export WHISPER_HIP_LIB=$GRAFT_REPO_ROOT/whisper.coreml_amd/lib/libwhisper_hip_tune.so
out=gpurun_out/rln_${tag}.txt
: > $out
for rep in 1 2; do
  for v in 1 0; do
    echo "RLN_256=$v" >> $out
    WHISPER_HIP_RLN_256=$v timeout -k 10 200 python3 -u profiles/xattn_probe.py large-v3 1,20 0 >> $out 2>&1 || exit 2
  done
done
cat $out
