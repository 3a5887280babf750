#!/bin/bash
# token-selection slice count at 100 rows (tuning library WHISPER_HIP_LP_NS): step graph ms
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ns in 0 16 32 0 16 32; do
  WHISPER_HIP_LIB=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so WHISPER_HIP_LP_NS=$ns \
    timeout -k 10 200 python3 profiles/step_profile.py --windows 20 --steps 32 | sed "s/^/ns $ns: /" >> gpurun_out/lp_ns_${tag}.txt 2>&1 || exit 1
done
cat gpurun_out/lp_ns_${tag}.txt
