#!/bin/bash
# cross-attention depth A/B (tuning library) + encoder PMC pass + HBM traffic PMC passes
#   profiles/session_run5.sh <tag>
set -o pipefail
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for d in 2 3 2 3; do
  echo "depth $d" >> gpurun_out/xdepth_${tag}.txt
  WHISPER_HIP_LIB=$PWD/whisper.coreml_amd/lib/libwhisper_hip_tune.so WHISPER_HIP_XS_DEPTH=$d \
    timeout -k 10 240 python3 profiles/xattn_probe.py large-v3 8,15,20,24 >> gpurun_out/xdepth_${tag}.txt 2>&1 || exit 1
done
cat gpurun_out/xdepth_${tag}.txt
bash profiles/enc_pmc.sh || exit 2
cat gpurun_out/enc_pmc.json | python3 -c "import json,sys; d=json.load(sys.stdin); [print(k, v.get('mean_ns'), v.get('mfma_busy_frac'), v.get('lds_conflict_frac')) for k,v in d.items()]"
bash profiles/pmc_pass.sh || exit 3
cat gpurun_out/traffic.json
